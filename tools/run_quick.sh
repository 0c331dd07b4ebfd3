set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in "MBK_RES32_PIX=128" "MBK_RES32_PIX=256 MBK_RES32_LDS_KB_SMALL=150" "MBK_RES32_PIX=64" "MBK_RES32_PIX=96 MBK_RES32_LDS_KB_SMALL=150"; do
  cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/lt
  env $v timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/lt -o run --output-format csv \
    -- python $GRAFT_REPO_ROOT/tools/learner_only.py --steps 2 > $GRAFT_REPO_ROOT/gpurun_out/r32.log 2>&1 || exit $?
  python $GRAFT_REPO_ROOT/tools/layer_times.py /tmp/lt --out $GRAFT_REPO_ROOT/gpurun_out/r32.md > /dev/null || exit $?
  echo "$v"; python $GRAFT_REPO_ROOT/tools/lt_agg.py $GRAFT_REPO_ROOT/gpurun_out/r32.md | grep "res_bwd32\|total"
done
