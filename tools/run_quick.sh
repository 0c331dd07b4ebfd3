set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
A="$GRAFT_REPO_ROOT/tools/learner_only.py --steps 1"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --kernel-trace -d /tmp/pa -o run --output-format csv -- python $A > $GRAFT_REPO_ROOT/gpurun_out/pa.log 2>&1 || exit 2
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC --kernel-trace -d /tmp/pb -o run --output-format csv -- python $A > $GRAFT_REPO_ROOT/gpurun_out/pb.log 2>&1 || exit 3
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace -d /tmp/pc -o run --output-format csv -- python $A > $GRAFT_REPO_ROOT/gpurun_out/pc.log 2>&1 || exit 4
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/pd -o run --output-format csv -- python $A > $GRAFT_REPO_ROOT/gpurun_out/pd.log 2>&1 || exit 5
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/pe -o run --output-format csv -- python $A > $GRAFT_REPO_ROOT/gpurun_out/pe.log 2>&1 || exit 6
python $GRAFT_REPO_ROOT/tools/pmc_raw.py "" /tmp/pa /tmp/pb /tmp/pc /tmp/pd /tmp/pe > $GRAFT_REPO_ROOT/gpurun_out/pmc_learner.txt
python $GRAFT_REPO_ROOT/tools/pmc_summary.py $GRAFT_REPO_ROOT/gpurun_out/pmc_learner.md /tmp/pb /tmp/pd /tmp/pe /tmp/pc > /dev/null 2>&1
ls -la $GRAFT_REPO_ROOT/gpurun_out/pmc_learner.*
