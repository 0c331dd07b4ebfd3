# Learner-path tests + one update's kernel trace (default knobs) + update timing.
#   bash tools/gpu_r4q.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4q}
timeout -k 10 400 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_fc.py tests/test_gpu_learner_parity.py tests/test_gpu_act.py tests/test_gpu_agent_api.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
bash tools/lt_ab.sh ${tag} "MBK_NOP=0" || exit 4
timeout -k 10 300 python tools/learner_only.py --steps 5 > gpurun_out/${tag}_learner.log 2>&1 || exit 3
echo "learner: $(tail -1 gpurun_out/${tag}_learner.log)"
