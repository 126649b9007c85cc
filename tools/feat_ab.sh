set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
for r in 1 2 3; do for l in base ntf; do
  ASTRO_LIB=$PWD/astro_amd/libastro_hip_$l.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-single --rollout 0 > gpurun_out/r6/feat_$l.json 2>/dev/null || exit 1
  python3 -c "
import json,sys; j=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); o=j['observation']; print(sys.argv[2], round(o['ms']*1e3,2), round(o['write_GBps']))" gpurun_out/r6/feat_$l.json $l | tee -a gpurun_out/r6/feat_ab.txt
done; done
