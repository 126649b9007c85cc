#!/usr/bin/env python3
"""Summarise tools/profile_r2.sh's rocprofv3 runs of one bench workload.

    python tools/prof_summary.py gpurun_out/r2prof/c3 c3

Writes, next to the runs:
  * traffic_<wl>_f32.json -- HBM bytes per one-tick astro_step launch:
    2 x FETCH_SIZE + WRITE_SIZE (KiB; MI355X_MICROARCH.md's gfx950
    correction: FETCH_SIZE counts 64 B per 128-B request of wide coalesced
    reads, so the read side is doubled);
  * pmc_<wl>_f32.json -- waves and VALU/SALU/f64 instructions per wave;
  * kernel_stats_<wl>.csv -- a copy of rocprofv3's kernel stats;
each tagged with the bench run's own workload state (mean live bullets,
resets per launch, from the JSON line the profiled run printed), which
bench.py checks before quoting them.  The one-tick step kernel is
astro_step_quad_kernel<..., MULTI = false, ...> or astro_step_kernel;
rollouts (MULTI = true) and the other kernels are left out.
"""
import csv
import json
import os
import shutil
import sys


def is_step(name):
    # demangled: astro_step_quad_kernel<float, 2, 4, false, 2, ...> (MULTI =
    # false); from round 5 the 9th argument is STATS: the timed region runs
    # the instance without counters (false), bench.py's counting pass the other
    if 'astro_step_quad_kernel<' in name:
        a = [x.strip() for x in name.split('<', 1)[1].split('>', 1)[0].split(',')]
        return a[3] == 'false' and (len(a) < 9 or a[8] == 'false')
    return 'astro_step_kernel<' in name


def bench_line(path):
    for line in open(path):
        line = line.strip()
        if line.startswith('{') and '"metric"' in line:
            return json.loads(line)
    raise SystemExit('no bench line in ' + path)


def counters(path, skip=10):
    acc = {}
    for r in csv.DictReader(open(path)):
        if is_step(r['Kernel_Name']):
            acc.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
    return {k: sum(v[skip:]) / len(v[skip:]) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    out, wl = sys.argv[1], sys.argv[2]
    b = bench_line(os.path.join(out, 'stats.log'))
    tag = dict(n_env=b['config']['n_env_per_gpu'], kernel=b['roofline']['kernel'],
               lanes_per_env=b['roofline']['lanes_per_env'],
               mean_live_bullets=b['stats']['mean_live_bullets'], resets_per_step=b['stats']['resets_per_step'],
               command='python bench.py %s (%s)' % (os.environ.get('PROFILE_ARGS', '--workload %s --no-cpu' % wl),
                                                   os.environ.get('PROFILE_SCRIPT', 'tools/profile_r2.sh')))
    tag['kernel'] = {1: 'lane', 2: 'pair', 4: 'quad'}[tag['lanes_per_env']]
    f, nf = counters(os.path.join(out, 'fetch', 'run_counter_collection.csv'))
    w, nw = counters(os.path.join(out, 'write', 'run_counter_collection.csv'))
    fetch, write = f['FETCH_SIZE'], w['WRITE_SIZE']
    traffic = dict(tag, launches=[nf['FETCH_SIZE'], nw['WRITE_SIZE']], fetch_size_kib=fetch,
                   write_size_kib=write, hbm_bytes_per_launch=(2 * fetch + write) * 1024,
                   algorithmic_bytes_per_launch=b['roofline']['bytes_per_launch'],
                   ratio=(2 * fetch + write) * 1024 / b['roofline']['bytes_per_launch'],
                   note='read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE; memory-side counters, '
                        'Infinity Cache hits included')
    rq = os.path.join(out, 'rdreq', 'run_counter_collection.csv')
    wq = os.path.join(out, 'wrreq', 'run_counter_collection.csv')
    if os.path.exists(rq) and os.path.exists(wq):
        # memory-side requests by size: reads of 32, 64 or 128 B; a write
        # request is 64 B (WRREQ_64B) or 32 B (the rest)
        r, _ = counters(rq)
        w2, _ = counters(wq)
        g = lambda d, k: next((v for n, v in d.items() if n.startswith(k) and n[len(k):] in ('', '_sum')), 0.0)
        n32, n64, n128 = g(r, 'TCC_EA0_RDREQ_32B'), g(r, 'TCC_EA0_RDREQ_64B'), g(r, 'TCC_EA0_RDREQ_128B')
        nw, nw64 = g(w2, 'TCC_EA0_WRREQ'), g(w2, 'TCC_EA0_WRREQ_64B')
        rd = 32 * n32 + 64 * n64 + 128 * n128
        wr = 64 * nw64 + 32 * (nw - nw64)
        traffic.update(rdreq=dict(total=g(r, 'TCC_EA0_RDREQ'), b32=n32, b64=n64, b128=n128),
                       wrreq=dict(total=nw, b64=nw64),
                       request_bytes_per_launch=rd + wr, request_read_bytes=rd, request_write_bytes=wr,
                       request_ratio=(rd + wr) / b['roofline']['bytes_per_launch'])
    json.dump(traffic, open(os.path.join(out, 'traffic_%s_f32.json' % wl), 'w'), indent=1)
    i, ni = counters(os.path.join(out, 'insts', 'run_counter_collection.csv'))
    wv = i['SQ_WAVES']
    pmc = dict(tag, waves=wv, valu_per_wave=i['SQ_INSTS_VALU'] / wv, salu_per_wave=i['SQ_INSTS_SALU'] / wv,
               f64_per_wave=(i['SQ_INSTS_VALU_MUL_F64'] + i['SQ_INSTS_VALU_ADD_F64']
                             + i['SQ_INSTS_VALU_FMA_F64']) / wv,
               launches=ni['SQ_WAVES'],
               note='a wave64 VALU instruction occupies its SIMD for 4 cycles: peak = 1024 SIMDs x '
                    '2.4 GHz / 4 = 614e9 wave-instructions/s')
    json.dump(pmc, open(os.path.join(out, 'pmc_%s_f32.json' % wl), 'w'), indent=1)
    src = os.path.join(out, 'stats', 'run_kernel_stats.csv')
    if os.path.exists(src):
        shutil.copy(src, os.path.join(out, 'kernel_stats_%s.csv' % wl))
    shutil.copy(os.path.join(out, 'stats.log'), os.path.join(out, 'bench_%s.log' % wl))
    print(json.dumps(dict(traffic=traffic['hbm_bytes_per_launch'], ratio=traffic['ratio'],
                          valu_per_wave=pmc['valu_per_wave'], bench_ms=b['ms_per_step'])))


if __name__ == '__main__':
    main()
