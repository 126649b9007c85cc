#!/usr/bin/env python3
"""Kernel-time sweep (HIP events per launch) over env count and features.

Diagnostic tool for the GPU box: prints one JSON line per variant with the
mean/median astro_step kernel time, env-steps/s of the kernel alone and the
steady-state stats.  All variants run interleaved-free but in ONE process
(same device, same clocks)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from astro_amd import BatchedEnv, DEFAULT_CONFIG  # noqa: E402
import bench  # noqa: E402


def run(name, cfg, n, ticks=200, warm=150, b_cap=32, p_pad=4, auto_reset=True, stats=True,
        dtype=torch.float32, kernel='auto'):
    env = BatchedEnv(cfg, n, device='cuda:0', b_cap=b_cap, p_pad=p_pad, dtype=dtype,
                     auto_reset=auto_reset, kernel=kernel)
    env.reset()
    ctl = torch.from_numpy(bench.controls(0, n, env.S, warm + ticks)).cuda()
    for t in range(warm):
        env.launch(ctl[t].data_ptr(), stats=stats)
    torch.cuda.synchronize()
    s0 = env.stat_dict()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(ticks)]
    st = torch.cuda.current_stream()
    for k in range(ticks):
        evs[k][0].record(st)
        env.launch(ctl[warm + k].data_ptr(), stats=stats)
        evs[k][1].record(st)
    torch.cuda.synchronize()
    ms = np.array([a.elapsed_time(b) for a, b in evs])
    s1 = env.stat_dict()
    d = {k: (s1[k] - s0[k]) / ticks for k in s0}
    print(json.dumps(dict(name=name, n=n, mean_us=ms.mean() * 1e3, med_us=float(np.median(ms)) * 1e3,
                          min_us=ms.min() * 1e3, env_steps_per_s=n / (ms.mean() * 1e-3),
                          bullets_per_env=d['bullets_in'] / n, resets=d['resets'],
                          planets_per_env=d['planets'] / n)), flush=True)


NSTAMP = 24   # the kernel's NSTAMP (stamp words per wave row)


def use_lib(name):
    from astro_amd import _lib
    _lib._lib = None
    _lib.load(os.path.join(ROOT, 'astro_amd', name))


def stamps(name, cfg, n, ticks=20, warm=150, b_cap=32, p_pad=4, lib='libastro_hip_stamps.so',
           kernel='lane', auto_reset=True):
    """Per-section cycle shares from the -DASTRO_STAMPS diagnostic library."""
    from astro_amd import _lib
    use_lib(lib)
    env = BatchedEnv(cfg, n, device='cuda:0', b_cap=b_cap, p_pad=p_pad, kernel=kernel, auto_reset=auto_reset)
    env.reset()
    nw = (n + 63) // 64 if kernel == 'lane' else ((n + 31) // 32 if kernel == 'pair' else (n + 15) // 16)
    ncr = 0
    env.stats = torch.zeros(nw + ncr, NSTAMP, dtype=torch.int64, device='cuda')
    ctl = torch.from_numpy(bench.controls(0, n, env.S, warm + ticks)).cuda()
    for t in range(warm):
        env.launch(ctl[t].data_ptr(), stats=False)
    rows = []
    for t in range(ticks):
        env.stats.zero_()
        env.launch(ctl[warm + t].data_ptr(), stats=True)
        torch.cuda.synchronize()
        rows.append(env.stats.cpu().numpy().astype(np.int64))
    R = np.stack(rows, 0)            # [ticks, nw + ncr, NSTAMP]
    C = R[:, nw:, :]                 # creator rows
    S = R[:, :nw, :].reshape(-1, NSTAMP)
    s0 = S[:, 0]
    tot = S[:, 11] - s0
    out = dict(name=name, n=n, wave_cycles_mean=float(tot.mean()), wave_cycles_max=float(tot.max()))
    def seg(a, b):
        ok = (S[:, a] > 0) & (S[:, b] > 0)
        return float((S[ok, b] - S[ok, a]).mean()) if ok.any() else None, float(ok.mean())
    for key, (a, b) in dict(hdr_wait=(0, 1), loads2_sincos_gravity=(1, 2), ship_collide=(2, 3),
                            bullets=(3, 4), reward=(4, 5), spawn_ships=(5, 6), planets=(6, 7),
                            chain_hdr=(7, 8), reset=(9, 10)).items():
        out[key] = seg(a, b)
    out['branches_total'] = float((S[:, 11] - S[:, 5]).mean())
    slow = tot >= np.percentile(tot, 90)
    Sm = S[slow]
    for key, (a, b) in dict(hdr_wait=(0, 1), loads2_sincos_gravity=(1, 2), ship_collide=(2, 3),
                            bullets=(3, 4), reward=(4, 5), branches=(5, 11)).items():
        out['slow10_' + key] = float((Sm[:, b] - Sm[:, a]).mean())
    out['slow10_total'] = float(tot[slow].mean())
    rt = (S[:, 13] - S[:, 12]).astype(np.float64)
    out['sclk_mhz'] = float((tot / np.maximum(rt, 1)).mean() * 100.0)
    out['wave_us_max'] = float(rt.max() / 100.0)
    out['wave_us_mean'] = float(rt.mean() / 100.0)
    # per launch: wave start / end relative to the launch's first wave start (100 MHz clock)
    rows_per = len(S) // ticks
    st_rel, en_rel = [], []
    for t in range(ticks):
        sl = slice(t * rows_per, (t + 1) * rows_per)
        t0w = S[sl, 12].min()
        st_rel.append((S[sl, 12] - t0w) / 100.0)
        en_rel.append((S[sl, 13] - t0w) / 100.0)
    st_rel, en_rel = np.concatenate(st_rel), np.concatenate(en_rel)
    out['wave_start_us'] = dict(mean=float(st_rel.mean()), p90=float(np.percentile(st_rel, 90)), max=float(st_rel.max()))
    out['wave_end_us'] = dict(mean=float(en_rel.mean()), p90=float(np.percentile(en_rel, 90)),
                              launch_mean=float(np.mean([e.max() for e in np.split(en_rel, ticks)])))
    if (S[:, 21] > 0).any():   # helper waves (HelpBox): posted -> done, relative to the launch's first wave
        hs, he = [], []
        for t in range(ticks):
            sl = slice(t * rows_per, (t + 1) * rows_per)
            t0w = S[sl, 12].min()
            ok = S[sl, 21] > 0
            hs.append((S[sl, 20][ok] - t0w) / 100.0)
            he.append((S[sl, 21][ok] - t0w) / 100.0)
        ends = [x.max() for x in he if x.size]
        out['helper_us'] = dict(seen_mean=float(np.concatenate(hs).mean()), end_mean=float(np.concatenate(he).mean()),
                                end_launch_mean=float(np.mean(ends)) if ends else None,
                                busy_frac=float((S[:, 22] > 0).mean()))
    if ncr:
        t0 = R[:, :nw, 12].min(1)[:, None].astype(np.float64)
        cs, cl, ce = [(C[:, :, k] - t0) / 100.0 for k in (0, 1, 2)]
        step_end = ((R[:, :nw, 13] - t0) / 100.0)
        out['creator_us'] = dict(start_mean=float(cs.mean()), start_max=float(cs.max()),
                                 last_flag_mean=float(cl.mean()), last_flag_max=float(cl.max()),
                                 end_mean=float(ce.mean()), end_max=float(ce.max()),
                                 step_end_max=float(step_end.max(1).mean()),
                                 served_mean=float(C[:, :, 3].mean()), batches_mean=float(C[:, :, 4].mean()))
        # publish (step wave slot 10) -> seen (creator slots 5..12) delay
        pub = R[:, :nw, 10].astype(np.float64)
        seen = C[:, :, 5:13].reshape(C.shape[0], -1)[:, :nw].astype(np.float64)
        ok = (pub > 0) & (seen > 0)
        dly = (seen - pub)[ok] / 100.0
        out['flag_delay_us'] = dict(mean=float(dly.mean()), p99=float(np.percentile(dly, 99)), max=float(dly.max()))
        pubrel = ((pub - t0) / 100.0)[ok]
        out['publish_us'] = dict(mean=float(pubrel.mean()), max=float(pubrel.max()))
    if kernel == 'quad':   # per-SIMD attribution (slots 14, 15 of the quad kernel's stamps)
        hw = S[:, 14] & 0xffffffff
        simd = ((S[:, 14] >> 32) << 16) | ((hw >> 4) & 0xfff)   # xcc | se, sh, cu, simd
        res, t0n, bul = S[:, 15] & 0xff, (S[:, 15] >> 8) & 0xff, (S[:, 15] >> 16) & 0xffff
        t_end = S[:, 13].astype(np.float64)
        rows = len(S) // ticks
        per = []
        for t in range(ticks):
            sl = slice(t * rows, (t + 1) * rows)
            keys, inv = np.unique(simd[sl], return_inverse=True)
            t0 = S[sl, 12].min()
            end = np.zeros(len(keys)); nres = np.zeros(len(keys)); nt0 = np.zeros(len(keys))
            nb = np.zeros(len(keys)); nw = np.zeros(len(keys))
            np.maximum.at(end, inv, (t_end[sl] - t0) / 100.0)
            np.add.at(nres, inv, res[sl]); np.add.at(nt0, inv, t0n[sl]); np.add.at(nb, inv, bul[sl])
            np.add.at(nw, inv, 1)
            per.append((end, nres, nt0, nb, nw))
        end = np.concatenate([x[0] for x in per]); nres = np.concatenate([x[1] for x in per])
        nt0 = np.concatenate([x[2] for x in per]); nb = np.concatenate([x[3] for x in per])
        nw = np.concatenate([x[4] for x in per])
        A = np.stack([np.ones_like(end), nres, nt0, nb / 64.0], 1)
        coef = np.linalg.lstsq(A, end, rcond=None)[0]
        out['simd_fit_us'] = dict(zip(['base', 'per_reset', 'per_t0', 'per_64_bullets'], coef.round(3).tolist()))
        out['simd_end_us'] = dict(mean=float(end.mean()), p99=float(np.percentile(end, 99)), max=float(end.max()))
        out['simd_waves'] = dict(mean=float(nw.mean()), max=float(nw.max()), min=float(nw.min()))
        top = end >= np.percentile(end, 99)
        out['simd_top1pct'] = dict(resets=float(nres[top].mean()), t0=float(nt0[top].mean()),
                                   bullets=float(nb[top].mean()), waves=float(nw[top].mean()))
        out['simd_all'] = dict(resets=float(nres.mean()), t0=float(nt0.mean()), bullets=float(nb.mean()))
    rs = S[:, 16:20].astype(np.float64)
    okr = (S[:, 9] > 0) & (S[:, 19] > 0)
    if okr.any():   # inside the (last) reset pass of a wave: chain + LDS, draws, create, stores
        r = S[okr]
        out['reset_parts'] = dict(chain=float((r[:, 16] - r[:, 9]).mean()), draws=float((r[:, 17] - r[:, 16]).mean()),
                                  create=float((r[:, 18] - r[:, 17]).mean()), stores=float((r[:, 19] - r[:, 18]).mean()),
                                  after=float((r[:, 10] - r[:, 19]).mean()))
    out['slow10_reset_share'] = float(((Sm[:, 9] > 0) & (Sm[:, 10] > 0)).mean())
    print(json.dumps(out), flush=True)
    _lib._lib = None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--set', default='basic')
    ap.add_argument('--libs', default='libastro_hip,libastro_hip_varB')
    a = ap.parse_args()
    D = DEFAULT_CONFIG
    if a.set == 'create':
        for n in (1024, 65536):
            env = BatchedEnv(D, n, device='cuda:0')
            env.reset()
            torch.cuda.synchronize()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
            for k in range(20):
                evs[k][0].record()
                env.reset()
                evs[k][1].record()
            torch.cuda.synchronize()
            ms = np.array([x.elapsed_time(y) for x, y in evs])
            seeds = np.arange(n, dtype=np.uint32) * 7919 + 13
            evs2 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
            st = torch.from_numpy(seeds.view(np.int32)).cuda()
            for k in range(20):
                evs2[k][0].record()
                env.reset(seeds=st)
                evs2[k][1].record()
            torch.cuda.synchronize()
            ms2 = np.array([x.elapsed_time(y) for x, y in evs2])
            print(json.dumps(dict(name='reset_stream', n=n, med_us=float(np.median(ms)) * 1e3,
                                  explicit_seed_med_us=float(np.median(ms2)) * 1e3)), flush=True)
        return
    if a.set == 'stub':
        for lib in a.libs.split(','):
            use_lib(lib + '.so')
            for k in ('lane', 'quad'):
                run(lib + ':' + k + ':c3', D, 65536, kernel=k)
                run(lib + ':' + k + ':c2', D._replace(reload_time=1000), 65536, kernel=k)
        return
    if a.set == 'kernels':
        for k in ('lane', 'quad'):
            run(k + ':c3', D, 65536, kernel=k)
            run(k + ':c3_noreset', D, 65536, auto_reset=False, kernel=k)
            run(k + ':c2', D._replace(reload_time=1000), 65536, kernel=k)
            run(k + ':c3_16k', D, 16384, kernel=k)
            run(k + ':c3_131k', D, 131072, kernel=k)
            run(k + ':c3_262k', D, 262144, kernel=k)
            run(k + ':c3_f64', D, 65536, dtype=torch.float64, kernel=k)
            run(k + ':c5', D._replace(max_planets=8), 131072, p_pad=8, kernel=k)
        return
    if a.set == 'epw':
        for lib in a.libs.split(','):
            use_lib(lib + '.so')
            run(lib + ':c3', D, 65536)
            run(lib + ':c2_noreset', D._replace(reload_time=1000), 65536, auto_reset=False)
            run(lib + ':c3_262k', D, 262144)
        return
    if a.set == 'timing':   # plain timings of alternative builds (-D A/B variants)
        for lib in a.libs.split(','):
            use_lib(lib + '.so')
            run(lib + ':c3', D, 65536)
            run(lib + ':c3_noreset', D, 65536, auto_reset=False)
        return
    if a.set == 'variants':
        for lib in a.libs.split(','):
            use_lib(lib + '.so')
            run(lib + ':c3', D, 65536)
            run(lib + ':c2', D._replace(reload_time=1000), 65536)
            run(lib + ':c3_noreset', D, 65536, auto_reset=False)
            stamps(lib + ':c3', D, 65536, lib=lib + '_stamps.so')
        return
    if a.set == 'c2':   # small-N layout study: c2 (4,096 envs, no bullets) and c3 for contrast
        c2 = D._replace(reload_time=1000)
        for k in ('quad', 'pair'):
            stamps(k + '_c2_4k', c2, 4096, kernel=k)
        stamps('quad_c2_4k_noreset', c2, 4096, kernel='quad', auto_reset=False)
        stamps('pair_c3', D, 65536, kernel='pair')
        return
    if a.set == 'stamps_pair':
        stamps('pair_c3', D, 65536, kernel='pair')
        stamps('quad_c3', D, 65536, kernel='quad')
        return
    if a.set == 'stamps':
        stamps('quad_c3', D, 65536, kernel='quad')
        stamps('quad_c2', D._replace(reload_time=1000), 65536, kernel='quad')
        stamps('c3', D, 65536)
        stamps('c2', D._replace(reload_time=1000), 65536)
        stamps('c3_16k', D, 16384)
        return
    if a.set == 'basic':
        for n in (16384, 65536, 262144, 1048576):
            run('c3', D, n)
        run('c3_nostats', D, 65536, stats=False)
        run('c3_noreset', D, 65536, auto_reset=False)
        run('c2_nobullets', D._replace(reload_time=1000), 65536)
        run('c2_nobullets_noreset', D._replace(reload_time=1000), 65536, auto_reset=False)
        run('c3_f64', D, 65536, dtype=torch.float64)
        run('c5', D._replace(max_planets=8), 131072, p_pad=8)


if __name__ == '__main__':
    main()
