set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s12
L=libastro_hip_base,libastro_hip_skip,libastro_hip_pin
for wl in c2 c3; do
  timeout -k 10 300 python tools/ab.py --libs $L --workload $wl > gpurun_out/s12/ab_$wl.jsonl 2>&1 || exit 1
done
timeout -k 10 300 python tools/sweep.py --set c2 > gpurun_out/s12/stamps.jsonl 2>gpurun_out/s12/stamps.err || { tail gpurun_out/s12/stamps.err; exit 1; }
cat gpurun_out/s12/ab_*.jsonl | grep -v amdgpu.ids | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'], d['n'], d['lib'][12:] or 'main', round(d['us_per_launch_median'], 3), round(d['rollout_us_per_tick'], 3))
"
python3 -c "
import json
for l in open('gpurun_out/s12/stamps.jsonl'):
    d=json.loads(l)
    print(d['name'], {k:(round(v[0]) if isinstance(v,list) and v[0] else v) for k,v in d.items() if k in ('hdr_wait','loads2_sincos_gravity','ship_collide','bullets','reward','spawn_ships','planets','chain_hdr','reset')}, d['wave_end_us'])
"
