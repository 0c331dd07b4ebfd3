# conv0_row queue (site 0) after the per-image refactor: tests, isolated learners, config-4 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread "$@" \
  > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 3; }
tail -1 gpurun_out/${tag}_pytest.log
for sz in "16 impala_flat 1" "24 impala_deep 0"; do set -- $sz
  for qv in 1 0; do
    timeout -k 10 300 python tools/learner_only.py --size $1 --arch $2 --bwd_occ $3 --active 0.023 --steps 5 --set native.mbk_set_work_queue_site=0:$qv \
      > gpurun_out/${tag}_lo.log 2>&1 || { tail -20 gpurun_out/${tag}_lo.log; exit 4; }
    echo "$1 $2 conv0 queue=$qv: $(tail -1 gpurun_out/${tag}_lo.log)"
  done
done
bash tools/gpu_r6_var2.sh ${tag}ab "1 2" "native.mbk_set_work_queue_site=0:0 -- --size 24 --arch impala_deep" "--size,24,--arch,impala_deep"
