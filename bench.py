#!/usr/bin/env python3
"""Batched lockstep Astro physics throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3]

One process per GPU (torchrun for N > 1).  Each rank steps its own shard of
envs (global env ids, no collective on the hot path); a "step" is one
astro_step launch = one tick of every env on that GPU, auto-reset included.
Controls are synthetic uniform random actions in [0, 6), keyed by (global
env id, tick) and resident in HBM before the timed region.  Rank 0 prints
one JSON line; value = env-steps of ALL ranks / max-over-ranks wall time.
"""
import argparse
import json
import multiprocessing as mp
import os
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=1000)
    ap.add_argument('--warmup', type=int, default=50)
    ap.add_argument('--workload', default='c3', choices=sorted(WORKLOADS))
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
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit('--gpus %d but WORLD_SIZE=%d' % (args.gpus, world))
    # one process per GPU; on a box with fewer GPUs than ranks (a rehearsal)
    # ranks share devices and ASTRO_DIST_BACKEND=gloo avoids RCCL's one-rank-per-GPU rule
    dev = torch.device('cuda', local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    backend = os.environ.get('ASTRO_DIST_BACKEND', 'nccl')
    red_dev = dev if backend == 'nccl' else None
    if world > 1:
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

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    for t in range(args.warmup):
        env.launch(ptrs[t])
    barrier()

    # Timed region: every one of the K launches has its own control buffer;
    # with --graph G they are captured G at a time into hipGraphs (capture
    # launches nothing) so the host's per-launch cost is out of the loop.
    graphs = []
    if args.graph > 0:
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(stream)
        with torch.cuda.stream(cap):
            for g0 in range(0, args.steps, args.graph):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=cap):
                    for k in range(g0, min(args.steps, g0 + args.graph)):
                        env.launch(ptrs[args.warmup + k])
                graphs.append(g)
        stream.wait_stream(cap)
    barrier()
    s0 = env.stat_dict()
    barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    if graphs:
        for g in graphs:
            g.replay()
    else:
        for k in range(args.steps):
            env.launch(ptrs[args.warmup + k])
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    barrier()
    s1 = env.stat_dict()
    gpu_ms_per_step = ev0.elapsed_time(ev1) / args.steps

    # Kernel duration: launches timed one by one (hipEvent pair around each,
    # on the launch stream), continuing the same games with fresh controls.
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.calib)]
    for k in range(args.calib):
        a, b = evs[k]
        a.record(stream)
        env.launch(ptrs[(args.warmup + k) % ticks])
        b.record(stream)
    torch.cuda.synchronize(dev)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))

    # Secondary lines (not the headline `value`).  (1) The same workload as
    # K-tick rollouts: controls from the on-device splitmix64 policy (the
    # same stream as `controls`), K ticks per launch, each wave stepping its
    # envs without a grid-wide barrier between ticks -- for open-loop or
    # scripted control, where no policy needs the observation between ticks.
    extras = {}
    if args.rollout > 0:
        K = args.rollout
        reps = max(1, args.steps // K)
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

    wall_max = _shard.max_over_ranks(wall, device=red_dev)
    d = {k: s1[k] - s0[k] for k in s0}
    fl = env.flags
    tot = _shard.sum_over_ranks([d[k] for k in ('bullets_in', 'resets', 'overflows', 'collisions',
                                                'timeouts')]
                                + [int(((fl & 1) != 0).sum()), int(((fl & 2) != 0).sum())], device=red_dev)
    # distinct devices behind the ranks (a one-GPU rehearsal shares one)
    n_dev = int(_shard.sum_over_ranks([1 if local < torch.cuda.device_count() else 0], device=red_dev)[0])
    bytes_launch = algorithmic_bytes(env, d, args.steps)

    if rank == 0:
        n_total = n * world
        value = n_total * args.steps / wall_max
        # per-launch duration = hipEvents bracketing the timed region (the
        # hipGraph replays) / K; rocprofv3's kernel average agrees within ~2%
        # (profiles/round1); one event pair per eager launch adds ~2.5 us
        launch_ms = gpu_ms_per_step
        achieved = bytes_launch / (launch_ms * 1e-3) / 1e9
        # PMC-measured HBM bytes and VALU instructions per launch come from
        # committed rocprofv3 runs of this same command (profiles/round2/);
        # they are used only when that run saw the same workload state
        # (envs, kernel, mean live bullets and resets per launch within 10%)
        mlb = tot[0] / (n_total * args.steps)
        rps = tot[1] / args.steps

        def matching(path):
            if not os.path.exists(path):
                return None
            with open(path) as f:
                j = json.load(f)
            ok = (j.get('n_env') == n and j.get('kernel') in (args.kernel, 'auto', env.step_kernel)
                  and abs(j.get('mean_live_bullets', -1) - mlb) <= 0.1 * max(mlb, 0.05) + 1e-9
                  and abs(j.get('resets_per_step', -1) - rps) <= 0.1 * max(rps, 1.0))
            return j if ok else None
        traffic = None
        tj = matching(args.traffic or os.path.join(ROOT, 'profiles', 'round2', 'traffic_%s_%s.json' % (
            args.workload, args.state)))
        if tj:
            traffic = tj.get('hbm_bytes_per_launch')
        # secondary bound: VALU issue, from the committed PMC instruction count
        # of this workload's kernel (profiles/round2/pmc_<workload>_<state>.json)
        issue = None
        pj = matching(os.path.join(ROOT, 'profiles', 'round2', 'pmc_%s_%s.json' % (args.workload, args.state)))
        if pj:
            lpe = dict(lane=1, quad=4, pair=2)[env.step_kernel]
            if pj.get('lanes_per_env') == lpe:
                rate = pj['waves'] * pj['valu_per_wave'] / (launch_ms * 1e-3)
                peak = 256 * 4 * 2.4e9 / 4
                issue = dict(bound='valu-issue', achieved=rate, peak=peak, unit='wave-instructions/s',
                             frac=rate / peak, valu_per_wave=pj['valu_per_wave'], waves=pj['waves'],
                             note='not HBM-bound and not issue-bound: two waves per SIMD at c3, '
                                  'latency-bound (DESIGN.md section 3)')
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
                          bytes_per_launch=bytes_launch, kernel_ms=launch_ms,
                          kernel_ms_eager_event_pairs=kern_ms,
                          kernel=('astro_step_kernel' if env.step_kernel == 'lane' else 'astro_step_quad_kernel'),
                          lanes_per_env=dict(lane=1, quad=4, pair=2)[env.step_kernel],
                          timing='hipEvent pair around the timed region / K launches'),
            issue_roofline=issue,
            gpu_ms_per_step=gpu_ms_per_step,
            timed_region='%d launches, %s' % (
                args.steps, ('replayed as %d hipGraph(s) of up to %d launches' % (len(graphs), args.graph))
                if graphs else 'launched eagerly'),
            burn_in_ticks=args.burn_in,
            stats=dict(mean_live_bullets=mlb,
                       serial_resets_per_step=d.get('serial_resets', 0) / args.steps,
                       resets_per_step=rps, overflow_bullets=tot[2],
                       collisions=tot[3], timeouts=tot[4],
                       mean_planets=d['planets'] / (n * args.steps),
                       envs_flag_overflow=tot[5], envs_flag_create_exhausted=tot[6]),
        )
        out.update(extras)
        if world == 1 and not args.no_cpu:
            procs = args.cpu_procs or cpu_share()
            out['cpu_baseline'] = cpu_baseline(wl['cfg'], args.cpu_seconds, procs, wl['planets_only'])
            out['speedup_vs_cpu'] = value / out['cpu_baseline']['value']
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
