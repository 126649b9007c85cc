#!/bin/bash
# concurrent shards on streams (tools/mb_streams.py), then the memory-kind GPU test
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/s2b; mkdir -p $OUT
timeout -k 10 300 python tools/mb_streams.py --shards 1,2,4 > $OUT/streams_auto.jsonl 2> $OUT/streams_auto.err
rc=$?; echo "streams auto rc=$rc"; cat $OUT/streams_auto.jsonl; [ $rc -ne 0 ] && { tail -5 $OUT/streams_auto.err; exit $rc; }
timeout -k 10 300 python tools/mb_streams.py --shards 2,4 --kernel pair > $OUT/streams_pair.jsonl 2> $OUT/streams_pair.err
rc=$?; echo "streams pair rc=$rc"; cat $OUT/streams_pair.jsonl; [ $rc -ne 0 ] && { tail -5 $OUT/streams_pair.err; exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_mem.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/test_mem.log 2>&1
rc=$?; echo "test_mem rc=$rc"; tail -3 $OUT/test_mem.log
exit $rc
