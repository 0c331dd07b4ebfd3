# Tiled learner scoring (mbk_head_score) vs head_fwd units: head tests, learner A/B, traces.
#   bash tools/gpu_r4l.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4l}
timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_learner_parity.py tests/test_gpu_act.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for v in 1 0; do
  MBK_HEAD_SCORE=$v timeout -k 10 300 python tools/learner_only.py --steps 5 > gpurun_out/${tag}_learner$v.log 2>&1 || exit 3
  echo "MBK_HEAD_SCORE=$v learner: $(tail -1 gpurun_out/${tag}_learner$v.log)"
done
bash tools/lt_ab.sh ${tag} "MBK_HEAD_SCORE=1" "MBK_HEAD_SCORE=0" || exit 4
grep -E "head_|update span" gpurun_out/${tag}_lt1.md gpurun_out/${tag}_lt2.md
