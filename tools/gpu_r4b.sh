# One GPU call: head / learner-parity tests, a learner kernel trace (layer_times table), then
# the acting-form A/B (tools/gpu_form_ab.sh: act tests + bench auto / fused / B).
#   bash tools/gpu_r4b.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4b}
timeout -k 10 400 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_learner_parity.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/${tag}_head_tests.log 2>&1 \
  || { tail -30 gpurun_out/${tag}_head_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_head_tests.log
bash tools/lt_ab.sh ${tag} "MBK_NOP=0" || exit 2
bash tools/gpu_form_ab.sh ${tag} || exit 3
