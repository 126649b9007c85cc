"""bench.py's own rank launcher, on CPU (gloo, a stub rank body).

``python bench.py --gpus N`` without torchrun starts N ranks itself (one
child per GPU with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*), so the driver's
multi-GPU run measures configs 4 and 5 however it is invoked.  ``--stub``
swaps the GPU body for the same process group, barrier and reductions."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = dict(os.environ, ASTRO_DIST_BACKEND='gloo', PYTHONDONTWRITEBYTECODE='1')
    env.pop('WORLD_SIZE', None)
    env.pop('RANK', None)
    env.pop('LOCAL_RANK', None)
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    lines = [l for l in p.stdout.splitlines() if l.strip().startswith('{')]
    return p, lines


def test_self_launched_ranks_print_one_line():
    p, lines = _run(['--gpus', '2', '--steps', '7', '--stub', '--no-cpu'])
    assert p.returncode == 0, p.stderr
    assert len(lines) == 1, p.stdout
    j = json.loads(lines[0])
    assert j['ranks'] == 2 and j['steps'] == 7 and j['stub']
    # max over ranks of the stub's per-rank wall (1 ms * (1 + rank))
    assert abs(j['ms_per_step'] - 2.0 / 7) < 1e-9


def test_multi_rank_line_carries_roofline_and_cpu_baseline():
    """BASELINE.json's metric is 'at 1/2/4/8 MI355X vs CPU core.step': a
    2-rank line carries the per-GPU roofline with an aggregate over ranks and
    the CPU baseline (rank 0, after every rank left the GPU region), through
    the same code path as a real rank."""
    p, lines = _run(['--gpus', '2', '--steps', '5', '--stub', '--cpu-seconds', '0.3', '--cpu-procs', '1'])
    assert p.returncode == 0, p.stderr
    j = json.loads(lines[0])
    assert {'roofline', 'cpu_baseline'} <= set(j)
    agg = j['roofline']['aggregate']
    # 2 ranks x 1000 stub bytes per launch x 5 launches / max wall (2 ms)
    assert abs(agg['achieved'] - 2 * 1000 * 5 / 0.002 / 1e9) < 1e-12
    cb = j['cpu_baseline']
    assert cb['cores'] == 1 and cb['kind'] == 'port' and cb['value'] > 0


def test_four_ranks_and_single_rank():
    p, lines = _run(['--gpus', '4', '--stub', '--no-cpu'])
    assert p.returncode == 0, p.stderr
    assert len(lines) == 1 and json.loads(lines[0])['ranks'] == 4
    p, lines = _run(['--gpus', '1', '--stub', '--no-cpu'])
    assert p.returncode == 0, p.stderr
    assert len(lines) == 1 and json.loads(lines[0])['ranks'] == 1


def test_failing_rank_ends_the_launch():
    """A rank that cannot join (bad backend name) fails the whole launch
    with a nonzero code instead of leaving the others waiting."""
    p, lines = _run(['--gpus', '2', '--stub', '--no-cpu'], {'ASTRO_DIST_BACKEND': 'no-such-backend'})
    assert p.returncode != 0
    assert lines == []


def test_counting_pass_skipped_on_device_errors():
    """With device error bits set by the timed region, bench.py's counting
    pass launches nothing and does not call stat_dict() (which raises on
    those bits), so the line still prints and reports them."""
    sys.path.insert(0, ROOT)
    import bench

    class FakeEnv:
        def stat_dict(self):
            raise AssertionError('stat_dict() called with device error bits set')

        def device_errors(self, clear=True):
            raise AssertionError('not expected')

    launched = []
    s0, s1 = {'resets': 1}, {'resets': 5}
    out = bench.counting_pass(FakeEnv(), launched.append, 20, s0, s1, 0x4, 0.0101)
    assert out == (s0, s1, 0.0101, 0x4) and launched == []


def test_region_breakdown_names_the_host_share():
    """bench.py's region_host_us: the host timestamps of the timed region,
    the launches' back-to-back GPU time, and -- when the event pair around
    the region was recorded -- the GPU's idle time inside it and the host's
    time after it."""
    sys.path.insert(0, ROOT)
    import bench
    st = dict(submitted=12.0, end_event_recorded=12.0, end_seen=12.5, synchronized=212.0)
    r = bench.region_breakdown(st, None, 0.0099, 20)
    assert abs(r['kernels_back_to_back'] - 198.0) < 1e-9
    assert abs(r['wall_minus_kernels_per_step'] - 0.7) < 1e-9
    assert 'gpu_span_events' not in r
    r = bench.region_breakdown(st, 0.0102, 0.0099, 20)
    assert abs(r['gpu_span_events'] - 204.0) < 1e-9 and abs(r['gpu_idle_in_span'] - 6.0) < 1e-9
    assert abs(r['host_after_gpu_span'] - 8.0) < 1e-9
