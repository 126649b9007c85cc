#!/usr/bin/env python3
"""HBM traffic per astro_step launch from rocprofv3 FETCH_SIZE / WRITE_SIZE
passes (tools/profile_round.sh), with the gfx950 correction of
MI355X_MICROARCH.md: FETCH_SIZE counts 64 B per 128-B request of wide
coalesced reads, so the read side is doubled; WRITE_SIZE is exact for
16-B-per-lane stores.  Both counters are in KiB.  Writes the JSON bench.py
reads as roofline.traffic."""
import csv
import json
import sys


def mean_counter(path, name, skip=20):
    v = [float(r['Counter_Value']) for r in csv.DictReader(open(path))
         if 'astro_step' in r['Kernel_Name'] and 'Lb1E' not in r['Kernel_Name']   # not rollouts
         and r['Counter_Name'] == name]
    v = v[skip:]
    return sum(v) / len(v), len(v)


fetch_csv, write_csv, out, n_env, kernel = sys.argv[1:6]
fetch, nf = mean_counter(fetch_csv, 'FETCH_SIZE')
write, nw = mean_counter(write_csv, 'WRITE_SIZE')
res = dict(n_env=int(n_env), kernel=kernel, launches=[nf, nw],
           fetch_size_kib=fetch, write_size_kib=write,
           hbm_bytes_per_launch=(2 * fetch + write) * 1024,
           note='read = 2 x FETCH_SIZE (gfx950 counts half of wide coalesced reads), write = WRITE_SIZE; '
                'working sets below 256 MiB fit the Infinity Cache, whose hits these '
                'memory-side counters include')
json.dump(res, open(out, 'w'), indent=1)
print(json.dumps(res))
