# PMC of the fp32 C2 LDS kernels side by side: k_lds_rows_dma (20,2) and k_lds_rows_rs (72,8)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-r06zb}; mkdir -p $OUT
for pl in "20 2" "72 8"; do
  t=$(echo $pl | tr ' ' x)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/lds_$t -o p -- python3 scripts/prof_one.py tblock_warp_total $pl f32 32 50 > $OUT/lds_$t.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/wait_$t -o p -- python3 scripts/prof_one.py tblock_warp_total $pl f32 32 50 > $OUT/wait_$t.log 2>&1 || exit 1
done
echo done
