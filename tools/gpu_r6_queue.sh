# learner work queues A/B: tests, isolated learner (queues on / off, bench cap), seed-paired bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" \
  > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 3; }
tail -1 gpurun_out/${tag}_pytest.log
for qv in 1 0; do
  timeout -k 10 200 python tools/learner_only.py --active 0.023 --steps 10 --bwd_occ 1 --set native.mbk_set_work_queues=$qv \
    > gpurun_out/${tag}_lo_$qv.log 2>&1 || { tail -20 gpurun_out/${tag}_lo_$qv.log; exit 4; }
  echo "queues=$qv: $(tail -1 gpurun_out/${tag}_lo_$qv.log)"
done
bash tools/gpu_r6_var2.sh ${tag}ab "${SEEDS:-1 2}" native.mbk_set_work_queues=0 base
