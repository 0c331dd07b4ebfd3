# weight-gradient work queue A/B: wgrad / encoder tests, isolated learner, seed-paired bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread "$@" \
  > gpurun_out/${tag}_pytest.log 2>&1; tail -4 gpurun_out/${tag}_pytest.log
for lib in new wq0; do la=""; [ $lib = wq0 ] && la="--lib variants/wq0"
  timeout -k 10 200 python tools/learner_only.py --active 0.023 --steps 10 --bwd_occ 1 $la > gpurun_out/${tag}_lo_$lib.log 2>&1 || { tail -20 gpurun_out/${tag}_lo_$lib.log; exit 4; }
  echo "$lib: $(tail -1 gpurun_out/${tag}_lo_$lib.log)"
done
bash tools/gpu_r6_var2.sh ${tag}ab "${SEEDS:-1 2 3}" lib=variants/wq0 base
