# Hardware-counter passes (one rocprofv3 run per pass, --kernel-trace for durations) of one
# command on the GPU box, summarised per kernel into gpurun_out/<name>_pmc.md.
#   bash tools/pmc.sh <name> <python args...>
# Pass 1: MFMA busy cycles + instruction count, LDS bank conflicts, GPU cycles (SQ x4, GRBM x1)
# Pass 2: FETCH_SIZE (TCC x3);  pass 3: WRITE_SIZE (TCC x2)  -> HBM bytes per kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
name=$1; shift
script=$1; shift
case $script in /*) ;; *) script=$R/$script ;; esac  # the passes run from /tmp
cd /tmp && export TMPDIR=/tmp
run() {  # run <dir> <counters...>
  local d=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d /tmp/${name}_$d -o run \
    --output-format csv -- python "${ARGS[@]}" > $R/gpurun_out/${name}_$d.log 2>&1
}
ARGS=("$script" "$@")
run p1 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE || exit 2
run p2 FETCH_SIZE || exit 3
run p3 WRITE_SIZE || exit 4
python $R/tools/pmc_summary.py $R/gpurun_out/${name}_pmc.md /tmp/${name}_p1 /tmp/${name}_p2 /tmp/${name}_p3
rm -rf /tmp/${name}_p1 /tmp/${name}_p2 /tmp/${name}_p3
