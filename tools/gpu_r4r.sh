# Headline bench A/B on one box, alternating: engine takes slots / publishes only once their
# learner-stream events executed (MBK_ENGINE_READY_ONLY=1, default) or behind a stream wait (0),
# with the learner head's compaction before the trunk (MBK_HEAD_PREP=1) or in the head (0).
#   bash tools/gpu_r4r.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4r}
timeout -k 10 400 python -u -m pytest tests/test_gpu_act.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
i=0
for rep in 1 2; do
for v in "MBK_ENGINE_READY_ONLY=1 MBK_HEAD_PREP=1" "MBK_ENGINE_READY_ONLY=1 MBK_HEAD_PREP=0" "MBK_ENGINE_READY_ONLY=0 MBK_HEAD_PREP=1" "MBK_ENGINE_READY_ONLY=0 MBK_HEAD_PREP=0"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/${tag}_b$i.log 2>&1 || exit 1
  echo "[$v] $(tail -1 gpurun_out/${tag}_b$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d["ms_per_step"])')"
done
done
