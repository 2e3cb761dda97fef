#!/bin/bash
# GPU box: batched learner parity (small-env shapes included), then the C4 A/B of the
# packed-lane agent phases (in-tree) against ab/libnopack.so.
set -o pipefail
OUT=gpurun_out/c4pack
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learn.py -x -q -k "philox_12x12 or odd_shapes or moore or config4 or trained_matches or coupled or async or curriculum or capture or episode_caps" --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab.sh "ab/libnopack.so ffm_amd/_lib/libffm_amd.so" --config 4 > $OUT/ab.log 2>&1 || { echo "ab failed"; tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
