set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rfE -s --timeout 300 --timeout-method thread -k "rock or Rock or fixed_count or packed or dist" > gpurun_out/pytest_rocket.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_rocket.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --kernels-only --profile-set rocket > gpurun_out/rocket_k.log 2>&1; rc=$?
echo "rocket rc=$rc"; tail -2 gpurun_out/rocket_k.log
