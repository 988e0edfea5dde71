set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rfE -s --timeout 300 --timeout-method thread -k "box or Box or pnqp or fused or packed or fixed_count or lqr_step or implicit or rock" > gpurun_out/pytest_sub.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_sub.log | tail -5
[ $rc -le 1 ] || exit $rc
bash tools/gpu_ab_multi.sh || exit 1
export DILQR_SKIP_BUILD_ID=1
for b in 0 100; do BOUNDS=$b timeout -k 10 200 python tools/phase_stamps.py 5 > gpurun_out/stamps_b$b.json || exit 1; echo "stamps $b: $(cat gpurun_out/stamps_b$b.json)"; done
bash tools/gpu_waves_exp.sh
