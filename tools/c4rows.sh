#!/bin/bash
# GPU box: the batched learner parity tests, then the C4 A/B against the HEAD build.
set -o pipefail
OUT=gpurun_out/c4rows
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learn.py -x -q -k "philox_12x12 or odd_shapes or moore or config4 or trained_matches or coupled or async" --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab.sh "ab/libhead.so ffm_amd/_lib/libffm_amd.so" --config 4 > $OUT/ab.log 2>&1 || { echo "ab failed"; tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
