# GPU test suite + headline bench + isolated microbench on the GPU box, stopping at the
# first crash / time limit (pytest rc 1 = test failures only: the bench still runs).
#   bash tools/gpu_suite.sh <tag> [extra pytest args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread "$@" \
  > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_bench.log | cut -c1-400
timeout -k 10 300 python tools/microbench.py --E 8192 --learn_B 8192 --iters 20 \
  > gpurun_out/${tag}_micro.log 2>&1 || exit $?
grep '"what"' gpurun_out/${tag}_micro.log | cut -c1-300
exit $rc
