# Round-2 measurement pass: counter calibration, enhance_128 forward-only HBM traffic, SQ
# (MFMA utilisation) for the forward / input-gradient / weight-gradient kernels, then the
# default bench line (with the CPU baseline) and its kernel-trace stats.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02}; mkdir -p $O
P="timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv"
BL="python3 tools/bench_layers.py --iters 3"
$P --pmc WRITE_SIZE -d $O/cal_write -o run -- tools/pmc_calib > $O/cal_write.log 2>&1
$P --pmc FETCH_SIZE -d $O/cal_fetch -o run -- tools/pmc_calib > $O/cal_fetch.log 2>&1
$P --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/cal_wrreq -o run -- tools/pmc_calib > $O/cal_wrreq.log 2>&1
echo calib done
$P --pmc FETCH_SIZE -d $O/e128_fetch -o run -- $BL --only enhance_128 --passes fwd > $O/e128_fetch.log 2>&1
$P --pmc WRITE_SIZE -d $O/e128_write -o run -- $BL --only enhance_128 --passes fwd > $O/e128_write.log 2>&1
$P --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/e128_wrreq -o run -- $BL --only enhance_128 --passes fwd > $O/e128_wrreq.log 2>&1
$P --pmc WRITE_SIZE -d $O/c0_write -o run -- $BL --only conv0_res --passes fwd > $O/c0_write.log 2>&1
$P --pmc FETCH_SIZE -d $O/wg_fetch -o run -- $BL --only enhance_128 --passes wgrad > $O/wg_fetch.log 2>&1
$P --pmc WRITE_SIZE -d $O/wg_write -o run -- $BL --only enhance_128 --passes wgrad > $O/wg_write.log 2>&1
echo traffic done
for pass in fwd dgrad wgrad; do
  $P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS \
    -d $O/sq_$pass -o run -- $BL --only enhance_128 --passes $pass > $O/sq_$pass.log 2>&1
  $P --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
    -d $O/sq2_$pass -o run -- $BL --only enhance_128 --passes $pass > $O/sq2_$pass.log 2>&1
done
echo sq done
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
echo bench done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline > $O/prof_bench.log 2>&1
echo all done
