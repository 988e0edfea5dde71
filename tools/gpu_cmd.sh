set -o pipefail
PYTEST_K="small_batch or next_cs or rocket or dense" bash tools/gpu_session_r05.sh || exit 1
AB_CMD=tools/ab_rocket_dense.py timeout -k 10 600 bash tools/ab.sh 3 > gpurun_out/ab_dense.txt 2>&1; rc=$?
cat gpurun_out/ab_dense.txt; exit $rc
