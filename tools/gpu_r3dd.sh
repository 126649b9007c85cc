#!/bin/bash
# host cost of a kernel launch (C microbenchmark; astro_step from Python and from C)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3dd
mkdir -p $O
timeout -k 10 120 ./tools/mb_hostlaunch > $O/mb_hostlaunch.jsonl 2>&1 || exit $?
cat $O/mb_hostlaunch.jsonl
timeout -k 10 200 python tools/host_launch_py.py > $O/host_launch_py.log 2>&1 || exit $?
tail -1 $O/host_launch_py.log
