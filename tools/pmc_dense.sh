set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
P=$R/tools/dense_pmc.py
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_dense_a -o run -- python3 $P > $R/gpurun_out/pmc_dense_a.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum --output-format csv -d $R/gpurun_out/pmc_dense_b -o run -- python3 $P > $R/gpurun_out/pmc_dense_b.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d $R/gpurun_out/pmc_dense_c -o run -- python3 $P > $R/gpurun_out/pmc_dense_c.log 2>&1
echo rc=$?
