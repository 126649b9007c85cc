#!/usr/bin/env python3
"""Batched lockstep Astro physics throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3]

One process per GPU: under torchrun (WORLD_SIZE set) this process is one
rank; with --gpus N > 1 and no launcher it starts the N ranks itself (one
child per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, RCCL) and never
touches the GPU.  Each rank steps its own shard of
envs (global env ids, no collective on the hot path); a "step" is one
astro_step launch = one tick of every env on that GPU, auto-reset included.
Controls are synthetic uniform random actions in [0, 6), keyed by (global
env id, tick) and resident in HBM before the timed region.  Rank 0 prints
one JSON line; value = env-steps of ALL ranks / max-over-ranks wall time.
"""
import argparse
import ctypes
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from astro_amd import BatchedEnv, DEFAULT_CONFIG  # noqa: E402
from astro_amd import shard as _shard  # noqa: E402

METRIC = 'env-steps/sec (batched lockstep) at 1/2/4/8 MI355X vs CPU core.step'
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)

# BASELINE.json configs 2, 3 and 5 (per GPU); configs 4 = c3 on 8 GPUs
WORKLOADS = {
    'c2': dict(n=4096, cfg=dict(reload_time=1000), b_cap=32, p_pad=4, planets_only=3,
               desc='4096 envs/GPU, DEFAULT_CONFIG with bullets disabled (reload_time=1000), '
                    '2 ships, 3 planets (generate_configs streams filtered to 3-planet games), '
                    'auto-reset, random actions'),
    'c3': dict(n=65536, cfg=dict(), b_cap=32, p_pad=4, planets_only=3,
               desc='65536 envs/GPU, DEFAULT_CONFIG (2 ships, 3 planets: generate_configs streams '
                    'filtered to 3-planet games; bullets on, b_cap 32 = 16/ship + overflow counter), '
                    'auto-reset, random actions'),
    'c3any': dict(n=65536, cfg=dict(), b_cap=32, p_pad=4, planets_only=0,
                  desc='65536 envs/GPU, DEFAULT_CONFIG unfiltered (2 ships, 1-4 planets), bullets on, '
                       'auto-reset, random actions'),
    'c5': dict(n=131072, cfg=dict(max_planets=8), b_cap=32, p_pad=8, planets_only=0,
               desc='131072 envs/GPU, DEFAULT_CONFIG with max_planets=8 (1-8 planets padded '
                    'to 8), bullets on, auto-reset, random actions'),
}


def controls(offset, n, nships, ticks, seed=0):
    """int8 [ticks, n, nships] uniform in [0, 6) from splitmix64(global id, tick)."""
    out = np.empty((ticks, n, nships), dtype=np.int8)
    ids = (np.arange(offset, offset + n, dtype=np.uint64)[:, None] * np.uint64(nships)
           + np.arange(nships, dtype=np.uint64)[None, :])
    with np.errstate(over='ignore'):
        for t in range(ticks):
            z = ids * np.uint64(0x9E3779B97F4A7C15) + np.uint64((t + 1) * 0xD1B54A32D192ED03 % (1 << 64)) \
                + np.uint64(seed)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            out[t] = ((z >> np.uint64(32)) * np.uint64(6) >> np.uint64(32)).astype(np.int8)
    return out


def _cpu_worker(args):
    cfg_kw, seconds, seed, planets_only = args
    from oracle import port
    return port.run_for(DEFAULT_CONFIG._replace(**cfg_kw), seconds, seed=seed, planets_only=planets_only)


def cpu_baseline(cfg_kw, seconds, procs, planets_only=0):
    """The single-game numpy port of core.step (oracle/port.py, pinned bit
    for bit to the reference) on `procs` host cores, one game per process."""
    if procs == 1:
        res = [_cpu_worker((cfg_kw, seconds, 0, planets_only))]
    else:
        with mp.get_context('spawn').Pool(procs) as pool:
            res = pool.map(_cpu_worker, [(cfg_kw, seconds, k, planets_only) for k in range(procs)])
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return dict(value=steps / wall, unit='env-steps/s', cores=procs, kind='port',
                sample='%d x %.0f s of single-game oracle/port.py step() (numpy restatement of '
                       'core.step, bit-exact to the reference), random actions, re-create on '
                       'termination%s: %d env-steps' % (procs, seconds, ' (3-planet games)' if planets_only else '',
                                                        steps),
                per_core=steps / wall / procs)


def cpu_share():
    """Host cores this process may use: OMP_NUM_THREADS when the launcher
    set it (the GPU box's per-GPU CPU share), else the affinity mask."""
    n = len(os.sched_getaffinity(0))
    try:
        omp = int(os.environ.get('OMP_NUM_THREADS', '0'))
    except ValueError:
        omp = 0
    return max(1, min(n, omp) if omp > 0 else n)


def algorithmic_bytes(env, dstats, launches):
    """SURVEY.md section 8(d)'s bytes per env-step, summed over a launch:
    2 * (20 S + 16 P + 16 B + 12) + S + 4 S + 1 -- header (3 words), ships
    (x, y, dx, dy, b), live planets and live bullets read and written, int8
    control in, float32 reward and uint8 done out -- with P and B the live
    planets and bullets the kernel's own counters saw (a bullet read,
    bullets_in, or written, bullets_out, counts once; 8-byte elements for
    float64 state)."""
    e = 8 if env.dtype == torch.float64 else 4
    S, N = env.S, env.n_env
    fixed = launches * N * (2 * (5 * e * S + 12) + S + 4 * S + 1)
    var = 2 * 4 * e * dstats['planets'] + 4 * e * (dstats['bullets_in'] + dstats['bullets_out'])
    return (fixed + var) / launches


def aggregate_roofline(bytes_all_ranks, steps, wall_max, n_dev):
    """Whole-job HBM roofline: every rank's section 8(d) bytes per launch,
    summed, times the launches, over the slowest rank's wall time, against
    the peak of the distinct GPUs behind the ranks."""
    peak = HBM_PEAK_GBS * max(1, n_dev)
    achieved = bytes_all_ranks * steps / wall_max / 1e9 if wall_max > 0 else 0.0
    return dict(achieved=achieved, peak=peak, unit='GB/s', frac=achieved / peak, n_gpus=n_dev,
                basis='sum over ranks of bytes per launch x launches / max-over-ranks wall (host clock, '
                      'the timed region)')


def add_cpu_baseline(out, wl, args):
    """The CPU baseline fields of the line (rank 0, after the GPU work)."""
    procs = args.cpu_procs or cpu_share()
    cb = cpu_baseline(wl['cfg'], args.cpu_seconds, procs, wl['planets_only'])
    world = out.get('ranks', 1)
    cb['host_share'] = ('rank 0\'s CPU share (%d of the job\'s %d GPU shares)' % (1, world) if world > 1
                        else 'the one GPU\'s CPU share')
    out['cpu_baseline'] = cb
    out['speedup_vs_cpu'] = out['value'] / cb['value'] if out['value'] else None
    out['speedup_basis'] = ('all %d ranks\' env-steps/s over one host share\'s CPU env-steps/s' % world if world > 1
                            else 'one GPU over its host share')


def single_game_latency(cfg, ticks=2000, seed=0, cpu=True):
    """The single-game drop-in (astro_amd.core, what astro/server.py's
    game_tick and core.play's loop call): us per core.step tick with random
    controls, re-creating on termination, and us per tick of core.play with
    two random bots (Bots.control + step + Tick bookkeeping); both arena
    modes of the shim, the default's numbers as the line's."""
    from astro_amd import core
    default = core.SHIM_MODE
    out = {}
    for mode in sorted(('mapped', 'copy'), key=lambda m: m == default):   # (the default last)
        core.clear_shims()
        core.SHIM_MODE = mode
        out.update(_single_game(core, cfg, ticks, seed))
        out['us_per_step_' + mode] = out['us_per_step']
    out['mode'] = default
    core.SHIM_MODE = default
    core.clear_shims()
    if not cpu:
        return out
    # the CPU comparison for this same path: oracle/port.py's core.step on
    # one host core, the same config, the same loop (controls drawn up front,
    # re-create on termination)
    from oracle import port
    g = port.Game(cfg)
    ctl = np.random.RandomState(seed).randint(0, 6, size=(ticks, 2))
    state = g.create(cfg.seed)
    t0 = time.perf_counter()
    for k in range(ticks):
        state, _ = g.step(state, ctl[k])
        if state is None:
            state = g.create(cfg.seed)
    out['cpu_port_us_per_step'] = (time.perf_counter() - t0) / ticks * 1e6
    out['cpu_port_sample'] = '%d core.step ticks of oracle/port.py on one host core, %s' % (
        ticks, 'DEFAULT_CONFIG' if cfg == DEFAULT_CONFIG else 'the same config')
    return out


def _single_game(core, cfg, ticks, seed):
    rng = np.random.RandomState(seed)
    state = core.create(cfg)
    for _ in range(50):   # first calls: the shim's buffers, the kernels' first launch
        state, _ = core.step(state, rng.randint(0, 6, size=2), cfg)
        if state is None:
            state = core.create(cfg)
    n_create = 0
    ctl = rng.randint(0, 6, size=(ticks, 2))   # (drawn up front, as the CPU comparison's loop)
    t0 = time.perf_counter()
    for k in range(ticks):
        state, _ = core.step(state, ctl[k], cfg)
        if state is None:
            state = core.create(cfg)
            n_create += 1
    dt = time.perf_counter() - t0
    bot = lambda s: int(rng.randint(0, 6))  # noqa: E731
    played = 0
    t1 = time.perf_counter()
    k = 0
    while played < ticks:
        g = core.play(cfg._replace(seed=k), [bot, bot])
        played += len(g.ticks)
        k += 1
    dp = time.perf_counter() - t1
    return dict(us_per_step=dt / ticks * 1e6, steps=ticks, creates=n_create, us_per_play_tick=dp / played * 1e6,
                play_ticks=played, games=k,
                path='astro_amd.core.step (float64 state, bit-exact to the reference): "mapped" (default): the '
                     'game in host memory the kernel addresses directly, a tick one astro_game_step call (pack, '
                     'launch, busy-wait, unpack in C); "copy": one H2D copy of the packed state, one launch, one D2H '
                     'copy, one event; the CPU reference port (oracle/port.py) per tick on one core beside it, the '
                     'same loop (controls drawn up front, re-create on termination)')


def region_breakdown(stamps, gpu_ms_stream, gpu_ms_per_step, steps):
    """Where the timed region's wall time went: the host timestamps
    (submitted = the launches or graph replays handed to the runtime,
    end_seen = the event behind them seen complete, synchronized = the
    clock's stop), the GPU's span of the region by the event pair around it
    (ev0 is recorded just before the clock starts, ev1 behind the launches),
    and the K launches' own back-to-back GPU time; the differences name the
    idle GPU time inside the region (first dispatch after the submission,
    graph overhead) and the host's tail (end poll, synchronize)."""
    out = {k: v for k, v in stamps.items()}
    kern = gpu_ms_per_step * steps * 1e3
    out['kernels_back_to_back'] = kern
    if gpu_ms_stream is not None:
        span = gpu_ms_stream * steps * 1e3
        out['gpu_span_events'] = span
        out['gpu_idle_in_span'] = span - kern
        out['host_after_gpu_span'] = stamps['synchronized'] - span
    out['wall_minus_kernels_per_step'] = (stamps['synchronized'] - kern) / steps
    return out


def counting_pass(env, launch, steps, s0, s1, dev_err, gpu_ms_per_step):
    """The K launches of the counting instance after the timed region
    (launch(k) issues the k-th): (s0, s1, gpu ms per launch, error bits).
    With device error bits already set (dev_err) nothing is launched and
    stat_dict(), which raises on them, is not called: the line still prints
    and reports the bits (device_errors), with the region's own s0/s1 and
    the counter-free GPU time standing in."""
    if dev_err:
        return s0, s1, gpu_ms_per_step, dev_err
    s0 = env.stat_dict()
    torch.cuda._sleep(int(2e6 + 4e4 * steps))
    q0e, q1e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    q0e.record()
    for k in range(steps):
        launch(k)
    q1e.record()
    torch.cuda.synchronize(env.device)
    dev_err |= env.device_errors(clear=False)
    s1 = env.stat_dict() if not dev_err else dict(s0)
    return s0, s1, q0e.elapsed_time(q1e) / steps, dev_err


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """--gpus N without a launcher: start N ranks of this script, one per
    GPU, as ``torch.distributed.run --nproc-per-node N`` would (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT); rank 0
    prints the line.  This process never initialises HIP (a parent that had
    would pass its GPU state to no one and hold a device context).  A rank
    that fails ends the others; the exit code is the first failure's."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:       # the rest would wait in a collective for ever
                    q.terminate()
        if live:
            time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def stub_rank(args, world, rank):
    """--stub: the rank body without a GPU (tests of the launcher on CPU):
    the same process group, barrier and max/sum-over-ranks reductions as a
    real rank, then rank 0's one JSON line."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group(os.environ.get('ASTRO_DIST_BACKEND', 'gloo'))
        dist.barrier()
    wall = _shard.max_over_ranks(0.001 * (1 + rank))
    n_ranks = int(_shard.sum_over_ranks([1])[0])
    bytes_all = float(_shard.sum_over_ranks([1000.0])[0])
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        out = dict(metric=METRIC, value=0.0, unit='env-steps/s', n_gpus=0, ranks=n_ranks,
                   steps=args.steps, warmup=args.warmup, ms_per_step=wall / max(1, args.steps) * 1e3,
                   higher_is_better=True, scaling='weak', vs_baseline=None, stub=True,
                   roofline=dict(bound='hbm', achieved=0.0, peak=HBM_PEAK_GBS, unit='GB/s', frac=0.0, traffic=None,
                                 scope='stub', aggregate=aggregate_roofline(bytes_all, args.steps, wall, n_ranks)))
        if not args.no_cpu:
            add_cpu_baseline(out, WORKLOADS[args.workload], args)
        print(json.dumps(out), flush=True)


PROFILE_ROUNDS = ('round6', 'round5', 'round4', 'round3', 'round2')
ROLLOUT_LAUNCHES = 10   # the rollout line's launches at least


def profile_file(name):
    """The newest committed profile of that name (profiles/round4, round3, then round2)."""
    for r in PROFILE_ROUNDS:
        p = os.path.join(ROOT, 'profiles', r, name)
        if os.path.exists(p):
            return p
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=1000)
    ap.add_argument('--warmup', type=int, default=50)
    ap.add_argument('--workload', default='c3', choices=sorted(WORKLOADS))
    ap.add_argument('--counters-in-region', action='store_true',
                    help='time the launches that count (stats rows) instead of counting in K further launches')
    ap.add_argument('--n-env', type=int, default=0, help='override envs per GPU')
    ap.add_argument('--state', default='f32', choices=['f32', 'f64'])
    ap.add_argument('--cpu-seconds', type=float, default=10.0)
    ap.add_argument('--cpu-procs', type=int, default=0,
                    help='host processes for the CPU baseline (0 = one per core of the '
                         "process's CPU share: OMP_NUM_THREADS if set, else its affinity mask)")
    ap.add_argument('--burn-in', type=int, default=300,
                    help='ticks every env plays (one astro_rollout launch, on-device random '
                         'controls) before the warmup, so the timed region sees steady-state '
                         'games (live bullets, resets) whatever --warmup is')
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--traffic', default='', help='JSON with PMC-measured HBM bytes per launch')
    ap.add_argument('--kernel', default='auto', choices=['auto', 'lane', 'quad', 'pair'])
    ap.add_argument('--graph', type=int, default=100,
                    help='launches per captured hipGraph in the timed region (0 = eager launches)')
    ap.add_argument('--calib', type=int, default=100,
                    help='eager launches timed one by one (hipEvent pairs) for the kernel duration')
    ap.add_argument('--rollout', type=int, default=100,
                    help='secondary line: the workload as K-tick rollouts with the on-device random '
                         'policy, K ticks per launch (0 = skip)')
    ap.add_argument('--no-features', action='store_true', help='skip the observation-builder line')
    ap.add_argument('--launcher', default='graph', choices=['graph', 'c'],
                    help='timed region: hipGraph replays of the captured launches, or the K launches issued '
                         'from C (astro_step_many)')
    ap.add_argument('--eager-head', type=int, default=0,
                    help='timed launches issued eagerly before the graph replays: the GPU runs them while the '
                         'host submits the first graph (~10-40 us), so it does not idle at the start of the region')
    ap.add_argument('--graph-first', type=int, default=0,
                    help='launches in the first captured graph (0 = --graph): a short first graph is '
                         'submitted quickly, so the GPU starts while the host submits the next')
    ap.add_argument('--host-warm-ms', type=float, default=0.0,
                    help='busy-wait the host this long right before the clock starts (the GPU is idle then)')
    ap.add_argument('--warm-ms', type=float, default=20.0,
                    help='untimed graph replays for this long (host ms) right before the timed region')
    ap.add_argument('--replay', default='raw', choices=['torch', 'raw'],
                    help="how the timed region replays a captured graph: hipGraphLaunch on its executable "
                         "graph directly (default: no per-replay wrapper; 20-step wall 14.75 -> 13.92 us median, "
                         "profiles/round3s2/ab_replay.jsonl), or torch's CUDAGraph.replay()")
    ap.add_argument('--end-poll', default='none', choices=['event', 'stream', 'none'],
                    help="how the host sees the region's end before its synchronize: nothing (default: "
                         "torch.cuda.synchronize alone, one marker round trip), busy-poll an event recorded behind "
                         "the launches (a second marker: +0.25 us per step at 20 steps, "
                         "profiles/round6/bench_end_poll.jsonl; the line then has the GPU span of the region), "
                         "or busy-poll the stream itself")
    ap.add_argument('--no-single', action='store_true', help='skip the single-game drop-in latency line')
    ap.add_argument('--stub', action='store_true', help=argparse.SUPPRESS)   # launcher test: no GPU work
    args = ap.parse_args()

    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit('--gpus %d but WORLD_SIZE=%d' % (args.gpus, world))
    if args.stub:
        return stub_rank(args, world, rank)
    # one process per GPU; on a box with fewer GPUs than ranks (a rehearsal)
    # ranks share devices and ASTRO_DIST_BACKEND=gloo avoids RCCL's one-rank-per-GPU rule
    dev = torch.device('cuda', local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    backend = os.environ.get('ASTRO_DIST_BACKEND', 'nccl')
    red_dev = dev if backend == 'nccl' else None
    # the process group: every multi-rank run, and a single rank when
    # ASTRO_DIST_INIT=1 (the RCCL initialisation, barrier and device-tensor
    # reductions of the multi-GPU path, exercised on one GPU)
    dist_on = world > 1 or os.environ.get('ASTRO_DIST_INIT', '') == '1'
    if dist_on:
        import torch.distributed as dist
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(backend)

    wl = WORKLOADS[args.workload]
    cfg = DEFAULT_CONFIG._replace(**wl['cfg'])
    n = args.n_env or wl['n']
    offset = rank * n
    env = BatchedEnv(cfg, n, device=dev, b_cap=wl['b_cap'], p_pad=wl['p_pad'],
                     dtype=torch.float64 if args.state == 'f64' else torch.float32,
                     env_offset=offset, auto_reset=True, kernel=args.kernel, planets_only=wl['planets_only'])
    env.reset()
    if args.burn_in > 0:   # age the batch: games of every age, bullets in flight
        env.rollout(args.burn_in, 'random', tick0=1 << 40, stats=False)
    ticks = args.warmup + args.steps
    ctl = torch.from_numpy(controls(offset, n, env.S, ticks)).to(dev)
    ptrs = [ctl[t].data_ptr() for t in range(ticks)]
    stream = torch.cuda.current_stream(dev)

    # the ranks' rendezvous: a host-side (gloo) group next to RCCL's, so a
    # barrier puts no collective kernel on the GPU right before the timed
    # region (the region follows the warm replays with nothing else between)
    bar_group = None
    if dist_on and backend == 'nccl':
        import torch.distributed as dist
        bar_group = dist.new_group(backend='gloo')

    def barrier():
        torch.cuda.synchronize(dev)
        if dist_on:
            import torch.distributed as dist
            dist.barrier(group=bar_group)

    # settle: a few eager launches of the one-tick instance after the burn-in's
    # rollout instance (the first launch after the switch is the slow one),
    # then the W warmup launches
    settle = 3
    cnt = args.counters_in_region   # (the region's launches: the build without the counters, unless asked)
    for t in range(settle):
        env.launch(ptrs[t % max(1, ticks)], stats=cnt)
    for t in range(args.warmup):
        env.launch(ptrs[t], stats=cnt)
    barrier()

    # Timed region: every one of the K launches has its own control buffer.
    # The first `eager_head` are launched eagerly, the rest were captured G at
    # a time into hipGraphs (capture launches nothing), so the host's
    # per-launch cost is out of the loop and the GPU runs the eager head while
    # the host submits the first graph.  Each graph is replayed once, untimed,
    # before the region: its first replay uploads it.
    head = min(args.steps, max(0, args.eager_head)) if args.graph > 0 else args.steps
    graphs, replays, graph_sizes = [], [], []
    use_c = args.launcher == 'c'
    if use_c:   # the K launches issued from C (astro_step_many), per-tick outputs
        head = 0
        rew_k = torch.empty(args.steps, n, env.S, dtype=torch.float32, device=dev)
        done_k = torch.empty(args.steps, n, dtype=torch.uint8, device=dev)
    if args.graph > 0 and head < args.steps and not use_c:
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(stream)
        with torch.cuda.stream(cap):
            bounds, g0 = [], head
            if args.graph_first > 0 and g0 < args.steps:   # a short first graph: submitted quickly
                bounds.append((g0, min(args.steps, g0 + args.graph_first)))
                g0 = bounds[-1][1]
            for g1 in range(g0, args.steps, args.graph):
                bounds.append((g1, min(args.steps, g1 + args.graph)))
            graph_sizes[:] = [b1 - b0 for b0, b1 in bounds]
            for b0, b1 in bounds:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=cap):
                    for k in range(b0, b1):
                        env.launch(ptrs[args.warmup + k], stats=cnt)
                graphs.append(g)
        stream.wait_stream(cap)
        replays = [g.replay for g in graphs]
        hgl = None
        if args.replay == 'raw' and graphs:
            # hipGraphLaunch of the HIP runtime the library (and torch) runs on,
            # resolved through the library's own dependency
            try:
                hgl = env.lib.hipGraphLaunch
            except AttributeError:   # (not resolvable: torch's replay, and the line says so)
                args.replay = 'torch'
        if hgl is not None:
            hgl.restype, hgl.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]
            sp = ctypes.c_void_p(stream.cuda_stream)

            def raw(ge):
                ge = ctypes.c_void_p(ge)

                def launch():
                    rc = hgl(ge, sp)
                    if rc != 0:
                        raise RuntimeError('hipGraphLaunch returned %d' % rc)
                return launch
            replays = [raw(g.raw_cuda_graph_exec()) for g in graphs]
        for r in replays:   # (the first replay uploads the graph)
            r()
        if not cnt:
            # the statistics at the region's start, read BEFORE the warm
            # replays: the launches they and the region run leave the stats
            # rows alone, and the region then follows the warm replays with
            # nothing but a synchronize in between (no reduction kernels or
            # copies: the same-process region A/B, tools/region_ab.py, times
            # 10.6-10.7 us per step back to back; after the stats read 11.2+)
            s0 = env.stat_dict()
        # keep the GPU busy for --warm-ms before the region, continuing the
        # games with the same graphs: on a box that idled before this process
        # the first short region ran at 20 us per step on the GPU's own
        # timeline, the next ones at 13 (profiles/round3s2/bench_c3_20_reps.jsonl).
        # Bounded on the GPU's progress, not the host's: each round of replays
        # is waited for before the next is queued, so at most one round is
        # in flight when the time is up
        t_w = time.perf_counter()
        ev_w = torch.cuda.Event()
        while time.perf_counter() - t_w < args.warm_ms * 1e-3:
            for r in replays:
                r()
            ev_w.record(stream)
            while not ev_w.query():
                pass
    if cnt or not graphs:
        barrier()
        s0 = env.stat_dict()
    barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    poll_event = args.end_poll == 'event'
    if poll_event:   # (instrumentation, before the clock starts: the GPU is idle, it runs at once)
        ev0.record(stream)
    if args.host_warm_ms > 0:   # (host only: the CPU core busy before the clock starts, the GPU idle)
        tw = time.perf_counter()
        while time.perf_counter() - tw < args.host_warm_ms * 1e-3:
            pass
    t0 = time.perf_counter()
    if use_c:
        env.launch_many(ptrs[args.warmup], args.steps, rew_k.data_ptr(), done_k.data_ptr(), stats=cnt)
    for k in range(head):
        env.launch(ptrs[args.warmup + k], stats=cnt)
    for r in replays:
        r()
    t_sub = time.perf_counter()
    if poll_event:
        ev1.record(stream)
        t_rec = time.perf_counter()
        while not ev1.query():   # (busy-poll the end: a blocking wait wakes ~10 us late)
            pass
    else:
        t_rec = t_sub
        while args.end_poll == 'stream' and not stream.query():
            pass
    t_end = time.perf_counter()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    # host timestamps inside the region (us from the clock's start)
    stamps = dict(submitted=(t_sub - t0) * 1e6, end_event_recorded=(t_rec - t0) * 1e6,
                  end_seen=(t_end - t0) * 1e6, synchronized=wall * 1e6)
    # faults of the timed region (read before stat_dict, which raises on them)
    dev_err = env.device_errors(clear=False)
    barrier()
    s1 = env.stat_dict() if not dev_err else dict(s0)
    gpu_ms_stream = ev0.elapsed_time(ev1) / args.steps if poll_event else None
    gpu_ms_graph = None
    if graphs:
        # The K launches' GPU time without the host's submission: the same
        # graphs replayed once more right after the region, the stream kept
        # busy by a ~1 ms spin kernel while the host submits them, the events
        # around the replays only (ROCm has no event nodes in graphs)
        torch.cuda._sleep(2000000)
        g0e, g1e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g0e.record(stream)
        for r in replays:
            r()
        g1e.record(stream)
        torch.cuda.synchronize(dev)
        gpu_ms_graph = g0e.elapsed_time(g1e) / (args.steps - head)
    # The launches' GPU time as the kernels run back to back: the K launches
    # issued eagerly (each its own AQL packet, no graph) behind a spin kernel
    # long enough for the host to submit them all, an event pair around them.
    # A graph replay adds ~15-20 us per graph on the GPU timeline (first node
    # behind the previous work), which a 20-launch run cannot amortise.
    torch.cuda._sleep(int(2e6 + 4e4 * args.steps))
    q0e, q1e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    q0e.record(stream)
    for k in range(args.steps):
        env.launch(ptrs[args.warmup + k], stats=cnt)
    q1e.record(stream)
    torch.cuda.synchronize(dev)
    gpu_ms_per_step = q0e.elapsed_time(q1e) / args.steps
    # The counters (live bullets and planets for the section 8(d) bytes,
    # resets, collisions, overflows): K more launches continuing the same
    # games, of the build that counts (stats rows; the timed region's
    # launches run without them, as a caller that passes no stats buffer
    # does), timed the same way for the record
    if not cnt:
        s0, s1, gpu_ms_counting, dev_err = counting_pass(
            env, lambda k: env.launch(ptrs[args.warmup + k], stats=True), args.steps, s0, s1,
            dev_err | env.device_errors(clear=False), gpu_ms_per_step)
    else:
        gpu_ms_counting = gpu_ms_per_step
    gpu_timing = ('%d launches issued back to back behind a spin kernel long enough for the host to submit them '
                  'all (right after the timed region, continuing its games): hipEvent pair / %d'
                  % (args.steps, args.steps))

    # Kernel duration: launches timed one by one (hipEvent pair around each,
    # on the launch stream), continuing the same games with fresh controls.
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.calib)]
    for k in range(args.calib):
        a, b = evs[k]
        a.record(stream)
        env.launch(ptrs[(args.warmup + k) % ticks], stats=cnt)
        b.record(stream)
    torch.cuda.synchronize(dev)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    # every launch since the region: the GPU-time replays and the calibration
    dev_err |= env.device_errors()

    # Secondary lines (not the headline `value`).  (1) The same workload as
    # K-tick rollouts: controls from the on-device splitmix64 policy (the
    # same stream as `controls`), K ticks per launch, each wave stepping its
    # envs without a grid-wide barrier between ticks -- for open-loop or
    # scripted control, where no policy needs the observation between ticks.
    extras = {}
    if args.rollout > 0:
        K = args.rollout
        # a fixed number of launches whatever --steps is (the driver's 20-step
        # run and a 1,000-step run time the same rollout region)
        reps = max(ROLLOUT_LAUNCHES, args.steps // K)
        base = ticks + args.calib
        env.rollout(K, 'random', tick0=base, stats=False)
        barrier()
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tr0 = time.perf_counter()
        r0.record(stream)
        for r in range(reps):
            env.rollout(K, 'random', tick0=base + (r + 1) * K, stats=False)
        r1.record(stream)
        torch.cuda.synchronize(dev)
        wall_r = _shard.max_over_ranks(time.perf_counter() - tr0, device=red_dev)
        barrier()
        extras['rollout'] = dict(
            ticks_per_launch=K, launches=reps, value=n * world * K * reps / wall_r, unit='env-steps/s',
            ms_per_tick=wall_r / (K * reps) * 1e3, gpu_ms_per_tick=r0.elapsed_time(r1) / (K * reps),
            policy='on-device splitmix64 random controls (bench controls stream)')
        # the same rollouts with script.ScriptBot deciding for both ships on
        # the device every tick (core.play's closed loop, core.py:377-410)
        env.rollout(K, 'script', tick0=base, stats=False)
        barrier()
        r0.record(stream)
        for r in range(reps):
            env.rollout(K, 'script', tick0=base + (r + 1) * K, stats=False)
        r1.record(stream)
        torch.cuda.synchronize(dev)
        barrier()
        sms = r0.elapsed_time(r1) / (K * reps)
        extras['rollout_script'] = dict(
            ticks_per_launch=K, launches=reps, gpu_ms_per_tick=sms, value=n * world * 1e3 / sms,
            unit='env-steps/s (GPU time)', policy='script.ScriptBot for every ship, decided on the device each tick')
    # (2) The observation builder (rl.ValueNetwork.get_features + to_batch):
    # an HBM-write-bound kernel; bytes = the float32 feature tensor written.
    if not args.no_features:
        out_f = env.features()
        torch.cuda.synchronize(dev)
        f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        f0.record(stream)
        for _ in range(20):
            env.features(out=out_f)
        f1.record(stream)
        torch.cuda.synchronize(dev)
        fms = f0.elapsed_time(f1) / 20
        fbytes = out_f.numel() * 4
        extras['observation'] = dict(
            kernel='astro_features_kernel', shape=list(out_f.shape), ms=fms,
            write_GBps=fbytes / (fms * 1e-3) / 1e9, hbm_frac=fbytes / (fms * 1e-3) / 1e9 / HBM_PEAK_GBS)

    dev_err |= env.device_errors()   # (the secondary lines' launches)
    wall_max = _shard.max_over_ranks(wall, device=red_dev)
    d = {k: s1[k] - s0[k] for k in s0}
    fl = env.flags
    tot = _shard.sum_over_ranks([d[k] for k in ('bullets_in', 'resets', 'overflows', 'collisions',
                                                'timeouts')]
                                + [int(((fl & 1) != 0).sum()), int(((fl & 2) != 0).sum()), dev_err],
                                device=red_dev)
    # distinct devices behind the ranks (a one-GPU rehearsal shares one)
    n_dev = int(_shard.sum_over_ranks([1 if local < torch.cuda.device_count() else 0], device=red_dev)[0])
    bytes_launch = algorithmic_bytes(env, d, args.steps)
    # every rank's section 8(d) bytes per launch, summed: the aggregate roofline
    bytes_all = float(_shard.sum_over_ranks([bytes_launch], device=red_dev)[0])

    if rank == 0:
        n_total = n * world
        value = n_total * args.steps / wall_max
        # per-launch duration = the K launches' GPU time / K (event-record
        # nodes inside the graphs: kernels plus the gaps between them, not the
        # host's submission); rocprofv3's kernel average is compared with it
        # in profiles/; one event pair per eager launch adds ~2.5 us
        launch_ms = gpu_ms_per_step
        achieved = bytes_launch / (launch_ms * 1e-3) / 1e9
        # PMC-measured HBM bytes and VALU instructions per launch come from
        # committed rocprofv3 runs of this same command (profiles/round2/);
        # they are used only when that run saw the same workload state
        # (envs, kernel, mean live bullets and resets per launch within 10%)
        mlb = tot[0] / (n_total * args.steps)
        rps = tot[1] / args.steps

        def matching(path, override=''):
            path = override or path
            if not path or not os.path.exists(path):
                return None
            with open(path) as f:
                j = json.load(f)
            j['_path'] = os.path.relpath(path, ROOT)
            ok = (j.get('n_env') == n and j.get('kernel') in (args.kernel, 'auto', env.step_kernel)
                  and abs(j.get('mean_live_bullets', -1) - mlb) <= 0.1 * max(mlb, 0.05) + 1e-9
                  and abs(j.get('resets_per_step', -1) - rps) <= 0.1 * max(rps, 1.0))
            return j if ok else None
        traffic = None
        tj = matching(profile_file('traffic_%s_%s.json' % (args.workload, args.state)), args.traffic)
        if tj:
            traffic = tj.get('hbm_bytes_per_launch')
        # secondary bound: VALU issue, from the committed PMC instruction count
        # of this workload's kernel (profiles/round*/pmc_<workload>_<state>.json).
        # SQ_WAVES / SQ_INSTS_VALU count every wave of the launch: with helper
        # waves (HelpBox) that is step and helper waves together, so the
        # per-launch total is what is compared with the issue peak, and the
        # per-wave figure is an average over both roles
        issue = None
        pj = matching(profile_file('pmc_%s_%s.json' % (args.workload, args.state)))
        if pj:
            lpe = dict(lane=1, quad=4, pair=2)[env.step_kernel]
            if pj.get('lanes_per_env') == lpe:
                valu_launch = pj['waves'] * pj['valu_per_wave']
                rate = valu_launch / (launch_ms * 1e-3)
                peak = 256 * 4 * 2.4e9 / 4
                sw, hw = env.launch_waves()
                per_simd = sw / 1024.0
                frac_i = rate / peak
                note = ('%d step waves (%.2f launched per SIMD)%s; %s' % (
                    sw, per_simd, (' + %d helper waves' % hw) if hw else '',
                    'issue-bound' if frac_i > 0.8 else
                    ('partly issue-bound: VALU issue %.0f%% of peak, the rest latency (DESIGN.md section 3)' % (
                        100 * frac_i) if frac_i > 0.45 else
                     'latency-bound: VALU issue %.0f%% of peak at %.1f waves per SIMD (DESIGN.md section 3)' % (
                         100 * frac_i, (sw + hw) / 1024.0))))
                issue = dict(bound='valu-issue', achieved=rate, peak=peak, unit='wave-instructions/s',
                             frac=frac_i, valu_per_launch=valu_launch,
                             f64_per_launch=pj['waves'] * pj.get('f64_per_wave', 0.0),
                             waves_counted=pj['waves'], step_waves=sw, helper_waves=hw,
                             valu_per_wave_both_roles=pj['valu_per_wave'], source=pj.get('_path'), note=note)
        out = dict(
            metric=METRIC, value=value, unit='env-steps/s', n_gpus=n_dev, ranks=world, steps=args.steps,
            warmup=args.warmup, ms_per_step=wall_max / args.steps * 1e3, higher_is_better=True,
            scaling='weak', vs_baseline=None,
            dtype='f64' if args.state == 'f64' else 'f64 math / f32 state',
            data='synthetic (random actions; games from generate_configs seed streams)',
            config=dict(workload='%s: %s' % (args.workload, wl['desc']), n_env_per_gpu=n,
                        n_env_total=n_total, b_cap=wl['b_cap'], p_pad=wl['p_pad'],
                        state=args.state, parallelism='env-shard x%d (no collectives)' % world),
            roofline=dict(bound='hbm', achieved=achieved, peak=HBM_PEAK_GBS, unit='GB/s',
                          frac=achieved / HBM_PEAK_GBS, traffic=traffic,
                          scope=('per GPU: rank 0\'s dominant kernel on its own GPU' if world > 1
                                 else 'the one GPU\'s dominant kernel'),
                          aggregate=aggregate_roofline(bytes_all, args.steps, wall_max, n_dev),
                          bytes_per_launch=bytes_launch, kernel_ms=launch_ms,
                          kernel_ms_eager_event_pairs=kern_ms,
                          kernel=('astro_step_kernel' if env.step_kernel == 'lane' else 'astro_step_quad_kernel'),
                          lanes_per_env=dict(lane=1, quad=4, pair=2)[env.step_kernel],
                          timing=gpu_timing),
            issue_roofline=issue,
            region_host_us=region_breakdown(stamps, gpu_ms_stream, gpu_ms_per_step, args.steps),
            gpu_ms_per_step=gpu_ms_per_step, gpu_ms_per_step_stream_events=gpu_ms_stream,
            gpu_ms_per_step_graph_replay=gpu_ms_graph,
            gpu_ms_per_step_counting=gpu_ms_counting,
            counters=('the timed launches' if cnt else
                      '%d further launches right after the timed region, continuing its games, of the instance that '
                      'counts (stats rows; the timed region runs the one without counters, as a caller passing no '
                      'stats buffer does): the stats below and the section 8(d) bytes per launch' % args.steps),
            timed_region=('%d launches issued from C in one astro_step_many call' % args.steps) if use_c else
                         '%d launches: %d eager, then %s' % (
                args.steps, head, ('%d hipGraph replay(s) of %s launches (%s), each graph replayed once '
                                   'untimed before the region' % (
                                       len(graphs), '+'.join(str(x) for x in graph_sizes),
                                       'hipGraphLaunch' if args.replay == 'raw' else 'torch CUDAGraph.replay'))
                if graphs else 'no graph'),
            dist=dict(initialized=dist_on, backend=backend if dist_on else None, world=world,
                      barrier=('host-side gloo group' if bar_group is not None else
                               (backend if dist_on else None)),
                      reductions='device tensors (RCCL all_reduce)' if dist_on and red_dev is not None
                      else ('host tensors (gloo)' if dist_on else 'none (one rank)')),
            burn_in_ticks=args.burn_in, settle_launches=settle, warm_ms=args.warm_ms,
            device_errors=int(tot[7]),
            stats=dict(mean_live_bullets=mlb,
                       serial_resets_per_step=d.get('serial_resets', 0) / args.steps,
                       resets_per_step=rps, overflow_bullets=tot[2],
                       collisions=tot[3], timeouts=tot[4],
                       mean_planets=d['planets'] / (n * args.steps),
                       envs_flag_overflow=tot[5], envs_flag_create_exhausted=tot[6]),
        )
        out.update(extras)
        if not args.no_single:   # (rank 0's own GPU; every rank is past the GPU region)
            out['single_game'] = single_game_latency(DEFAULT_CONFIG, cpu=not args.no_cpu)
    # rank 0's host-side lines run after every rank has left the GPU region
    # (the last collective above): the CPU baseline of the same workload, on
    # this rank's CPU share, for any number of ranks
    if dist_on:
        import torch.distributed as dist
        dist.destroy_process_group()
    if rank == 0:
        if not args.no_cpu:
            add_cpu_baseline(out, wl, args)
        print(json.dumps(out), flush=True)
        if int(tot[7]):
            raise SystemExit('bench: a launch reported device error bits (device_errors=%d): the state '
                             'and the line above are not trusted' % int(tot[7]))


if __name__ == '__main__':
    sys.exit(main() or 0)
