#!/bin/bash
# GPU box, end of the session's work: full GPU suite + smoke + bench lines and traces
# (tools/final_check.sh), then PMC HBM traffic of the C2 and C5 step kernels.
set -o pipefail
TAG=${1:-r02_final}
bash tools/final_check.sh $TAG || exit 1
bash tools/traffic.sh gpurun_out/$TAG/traffic_c2 > gpurun_out/$TAG/traffic_c2.log 2>&1 || { tail gpurun_out/$TAG/traffic_c2.log; exit 1; }
cat gpurun_out/$TAG/traffic_c2/traffic.json
bash tools/traffic.sh gpurun_out/$TAG/traffic_c5 --config 5 > gpurun_out/$TAG/traffic_c5.log 2>&1 || { tail gpurun_out/$TAG/traffic_c5.log; exit 1; }
cat gpurun_out/$TAG/traffic_c5/traffic.json
