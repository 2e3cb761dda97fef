#!/bin/bash
# GPU box: the large-placement test, then the learner suite's reset / tiled / config-5 tests.
set -o pipefail
OUT=gpurun_out/place
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learn.py -x -v -k "large_placement or tiled_step or config5 or owner_shards or episode_caps or large_rooms" --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
