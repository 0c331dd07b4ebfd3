# stage-0 pool-fused weight gradient with 1 image per round (36 KB: two workgroups per CU
# beside an acting one) vs 2: tests, isolated learner at the bench cap, seed-paired bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread "$@" \
  > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 3; }
tail -1 gpurun_out/${tag}_pytest.log
for v in 2 1; do
  timeout -k 10 200 python tools/learner_only.py --active 0.023 --steps 10 --bwd_occ 1 --set enc.wgrad0_imgs=$v \
    > gpurun_out/${tag}_lo_$v.log 2>&1 || { tail -20 gpurun_out/${tag}_lo_$v.log; exit 4; }
  echo "wgrad0_imgs=$v: $(tail -1 gpurun_out/${tag}_lo_$v.log)"
done
bash tools/gpu_r6_var2.sh ${tag}ab "${SEEDS:-1 2 3}" base wgrad0_imgs=1
