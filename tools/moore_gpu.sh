set -o pipefail
mkdir -p gpurun_out/moore
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learn.py -x -v -k "moore" --timeout 600 --timeout-method thread > gpurun_out/moore/moore.log 2>&1 || { echo "moore failed"; tail -40 gpurun_out/moore/moore.log; exit 1; }
tail -3 gpurun_out/moore/moore.log
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/moore/suite.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/moore/suite.log; exit 1; }
tail -3 gpurun_out/moore/suite.log
