#!/usr/bin/env python3
"""Per-section cycles of one step-wave launch from the -DASTRO_STAMPS build
(tools/build_var.sh stamps ... -DASTRO_STAMPS): s_memtime stamps at section
boundaries, one row per step wave (stats buffer), averaged over launches
after a burn-in.  Round 3 adds stamps inside the bullet pass (16: bodies in
LDS, 17: first rounds done) and after bullets_begin (19).
    python tools/stamps_r3.py --workload c3 [--lib libastro_hip_stamps]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from astro_amd import BatchedEnv, DEFAULT_CONFIG, _lib  # noqa: E402

NSTAMP = 36
SEGS = dict(hdr_wait=(0, 1), bullets_begin=(1, 19), sincos_gravity=(19, 2), ship_collide=(2, 3),
            bodies_lds=(3, 16), rounds_first=(16, 17), rounds_rest=(17, 4), reward_post=(4, 5),
            spawn_ships=(5, 6), planets=(6, 7), hdr_store=(7, 8))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', default='c3')
    ap.add_argument('--lib', default='libastro_hip_stamps')
    ap.add_argument('--ticks', type=int, default=20)
    ap.add_argument('--warm', type=int, default=300)
    ap.add_argument('--b2b', action='store_true',
                    help='the measured launches back to back (one stats buffer each, one sync at the end): '
                         'adds the gap between a launch\'s last wave and the next launch\'s first')
    ap.add_argument('--timing-only', action='store_true')
    a = ap.parse_args()
    _lib._lib = None
    _lib.load(os.path.join(ROOT, 'astro_amd', a.lib + '.so'))
    w = bench.WORKLOADS[a.workload]
    n = w['n']
    env = BatchedEnv(DEFAULT_CONFIG._replace(**w['cfg']), n, device='cuda:0', b_cap=w['b_cap'], p_pad=w['p_pad'],
                     auto_reset=True, planets_only=w['planets_only'])
    env.reset()
    lpe = dict(lane=1, quad=4, pair=2)[env.step_kernel]
    nw = (n * lpe + 63) // 64
    env.stats = torch.zeros(nw, NSTAMP, dtype=torch.int64, device='cuda')
    env.rollout(a.warm, 'random', tick0=1 << 40, stats=False)
    ctl = torch.from_numpy(bench.controls(0, n, env.S, a.ticks + 5)).cuda()
    for t in range(5):
        env.launch(ctl[t].data_ptr(), stats=False)
    rows = []
    if a.b2b:
        bufs = [torch.zeros(nw, NSTAMP, dtype=torch.int64, device='cuda') for _ in range(a.ticks)]
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for t in range(a.ticks):
            env.stats = bufs[t]
            env.launch(ctl[5 + t].data_ptr(), stats=True)
        e1.record()
        torch.cuda.synchronize()
        b2b_event_us = e0.elapsed_time(e1) * 1e3 / a.ticks
        rows = [b.cpu().numpy().astype(np.int64) for b in bufs]
    else:
        for t in range(a.ticks):
            env.stats.zero_()
            env.launch(ctl[5 + t].data_ptr(), stats=True)
            torch.cuda.synchronize()
            rows.append(env.stats.cpu().numpy().astype(np.int64))
    if a.timing_only:   # (a build without stamps: the event timing of the same launches only)
        print(json.dumps(dict(workload=a.workload, lib=a.lib, b2b_event_us=b2b_event_us)), flush=True)
        return
    S = np.concatenate(rows, 0)
    tot = S[:, 11] - S[:, 0]
    out = dict(workload=a.workload, n=n, kernel=env.step_kernel, waves=nw, wave_cycles_mean=float(tot.mean()))
    for k, (x, y) in SEGS.items():
        ok = (S[:, x] > 0) & (S[:, y] > 0)
        out[k] = [round(float((S[ok, y] - S[ok, x]).mean()), 1), round(float(ok.mean()), 3)] if ok.any() else None
    rt = (S[:, 13] - S[:, 12]).astype(np.float64)
    out['sclk_mhz'] = float((tot / np.maximum(rt, 1)).mean() * 100.0)
    st, en = [], []
    for t in range(a.ticks):
        R = S[t * nw:(t + 1) * nw]
        t0 = R[:, 12].min()
        st.append((R[:, 12] - t0) / 100.0)
        en.append((R[:, 13] - t0) / 100.0)
    out['wave_start_us_mean'] = float(np.concatenate(st).mean())
    out['wave_end_us_mean'] = float(np.concatenate(en).mean())
    out['launch_last_wave_end_us'] = float(np.mean([e.max() for e in en]))
    # every launch's first wave start and last wave end (step or helper) on
    # the 100 MHz real-time clock: with --b2b the time between launches
    first = [int(S[t * nw:(t + 1) * nw, 12].min()) for t in range(a.ticks)]
    last = []
    for t in range(a.ticks):
        R = S[t * nw:(t + 1) * nw]
        e = int(R[:, 13].max())
        if (R[:, 21] > 0).any():
            e = max(e, int(R[R[:, 21] > 0, 21].max()))
        last.append(e)
    if a.b2b:
        span = [(last[t] - first[t]) / 100.0 for t in range(a.ticks)]
        gap = [(first[t + 1] - last[t]) / 100.0 for t in range(a.ticks - 1)]
        per = [(first[t + 1] - first[t]) / 100.0 for t in range(a.ticks - 1)]
        out['b2b'] = dict(event_us_per_launch=b2b_event_us, span_us_mean=float(np.mean(span)), gap_us_mean=float(np.mean(gap)),
                          gap_us_min=float(np.min(gap)), period_us_mean=float(np.mean(per)))
    if (S[:, 21] > 0).any():
        he = []
        for t in range(a.ticks):
            R = S[t * nw:(t + 1) * nw]
            t0 = R[:, 12].min()
            ok = R[:, 21] > 0
            he.append(((R[ok, 21] - t0) / 100.0).max() if ok.any() else 0.0)
        out['helper_last_end_us'] = float(np.mean(he))
        # the helpers after the post: stamp 20 = post seen, 21 = end (both
        # s_memrealtime), 22 = finished envs posted
        ok = (S[:, 20] > 0) & (S[:, 21] > 0)
        nr = S[:, 22]
        aft = (S[:, 21] - S[:, 20]) / 100.0
        out['helper_after_post_us'] = {str(k): [round(float(aft[ok & (np.minimum(nr, 2) == k)].mean()), 3),
                                               int((ok & (np.minimum(nr, 2) == k)).sum())]
                                       for k in (0, 1, 2) if (ok & (np.minimum(nr, 2) == k)).any()}
        post = []
        for t in range(a.ticks):
            R = S[t * nw:(t + 1) * nw]
            t0 = R[:, 12].min()
            okr = R[:, 20] > 0
            post.append(((R[okr, 20] - t0) / 100.0).mean() if okr.any() else 0.0)
        out['helper_post_seen_us_mean'] = float(np.mean(post))
        # of the launch's 1% last-ending helpers: how many had resets
        ends = []
        for t in range(a.ticks):
            R = S[t * nw:(t + 1) * nw]
            okr = R[:, 21] > 0
            e = R[okr, 21]
            cut = np.percentile(e, 99)
            ends.append(float((R[okr][e >= cut, 22] > 0).mean()))
        out['helper_top1pct_with_resets'] = float(np.mean(ends))
    # the helper wave's own sections (s_memtime stamps 24-30, shader cycles),
    # by the number of finished games it re-created
    if (S[:, 30] > 0).any():
        hseg = dict(hdr_chains=(24, 25), planet_update=(25, 26), wait_post=(26, 27), survivor_stores=(27, 28),
                    reset_passes=(28, 29), tail=(29, 30), total=(24, 30),
                    # the last reset pass's sections (wave_reset_pass stamps 16-19, copied to 32-35)
                    pass_shuffles_temper=(28, 32), pass_draws=(32, 33), pass_create=(33, 34), pass_stores=(34, 35))
        nr = np.minimum(S[:, 22], 2)
        hout = {}
        for k, (x, y) in hseg.items():
            d = (S[:, y] - S[:, x]).astype(np.float64)
            row = {}
            for r in (0, 1, 2):
                ok = (S[:, x] > 0) & (S[:, y] > 0) & (nr == r)
                if ok.any():
                    row[str(r)] = round(float(d[ok].mean()), 1)
            hout[k] = row
        out['helper_cycles_by_resets'] = hout
        st0 = []
        for t in range(a.ticks):
            R = S[t * nw:(t + 1) * nw]
            t0 = R[:, 12].min()
            ok = R[:, 23] > 0
            st0.append(((R[ok, 23] - t0) / 100.0).mean() if ok.any() else 0.0)
        out['helper_start_us_mean'] = float(np.mean(st0))
    # what makes a wave slow: its live bullets, games at their first tick,
    # finished games (stamp 15 = resets | t0 << 8 | bullets << 16)
    info = S[:, 15]
    nres, nt0, nbul = info & 0xff, (info >> 8) & 0xff, (info >> 16) & 0xffff
    cyc = tot.astype(np.float64)
    slow = cyc >= np.percentile(cyc, 95)
    out['slow5'] = dict(cycles=float(cyc[slow].mean()), bullets=float(nbul[slow].mean()), t0=float(nt0[slow].mean()),
                        resets=float(nres[slow].mean()), start_us=float(np.concatenate(st)[slow].mean()))
    out['all'] = dict(cycles=float(cyc.mean()), bullets=float(nbul.mean()), t0=float(nt0.mean()), resets=float(nres.mean()))
    # a step wave's own (last) reset pass (no helper waves): stamps 16-19 are
    # the pass's there (they overwrite the bullet pass's 16, 17 and 19)
    rs = (nres > 0) & (S[:, 16] > 0) & (S[:, 19] > 0)
    if rs.any() and not (S[:, 30] > 0).any():
        st_pass = np.maximum(S[:, 8], S[:, 9])
        out['step_pass_cycles'] = dict(
            waves=int(rs.sum()), before_draws=float((S[rs, 16] - st_pass[rs]).mean()),
            draws=float((S[rs, 17] - S[rs, 16]).mean()), create=float((S[rs, 18] - S[rs, 17]).mean()),
            stores=float((S[rs, 19] - S[rs, 18]).mean()), after=float((S[rs, 10] - S[rs, 19]).mean()))
    A = np.stack([np.ones_like(cyc), nbul, nt0, nres], 1).astype(np.float64)
    coef = np.linalg.lstsq(A, cyc, rcond=None)[0]
    out['fit_cycles'] = dict(base=float(coef[0]), per_bullet=float(coef[1]), per_t0=float(coef[2]), per_reset=float(coef[3]))
    for k in SEGS:
        x, y = SEGS[k]
        ok = (S[:, x] > 0) & (S[:, y] > 0)
        if ok.any():
            d = (S[:, y] - S[:, x]).astype(np.float64)
            out.setdefault('slow5_seg', {})[k] = round(float(d[slow & ok].mean()), 1) if (slow & ok).any() else None
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
