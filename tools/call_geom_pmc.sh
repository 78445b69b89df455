# Why 1024-thread map blocks win: PMC passes per map geometry,
# then the exact RCCL message for two ranks on one GPU (item 3).
export TMPDIR=/tmp
PMC="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS" \
  bash tools/pmc_variants.sh > gpurun_out/geom_pmc1.txt 2>&1 || { cat gpurun_out/geom_pmc1.txt; exit 1; }
PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
  bash tools/pmc_variants.sh > gpurun_out/geom_pmc2.txt 2>&1 || { cat gpurun_out/geom_pmc2.txt; exit 1; }
cat gpurun_out/geom_pmc1.txt gpurun_out/geom_pmc2.txt
NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT bash tools/rccl_one_gpu.sh --steps 5 --warmup 1 > gpurun_out/rccl1g_info.txt 2>&1
echo rccl_rc=$?
grep -h -i -E "warn|duplicate|same|invalid|error" gpurun_out/rccl1g_rank*.out gpurun_out/rccl1g_rank*.err | head -30
