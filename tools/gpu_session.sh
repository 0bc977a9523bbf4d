#!/bin/bash
# tools/gpu_session.sh STEP... -- run on the GPU box (via gpurun) from the repo root.
# Each step runs under its own timeout; a crash/timeout (exit not in {0,1}) ends
# the session immediately (no further GPU work in this call).
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session.log
  local s=$(date +%s)
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - s ))s)" | tee -a $OUT/session.log
  tail -5 $OUT/$name.log | sed 's/^/    /'
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    info) run info 60 bash -c "rocm-smi --showproductname --showclocks 2>&1 | head -40; nproc; lscpu | grep 'Model name'" ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    test) run pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    testall) run pytest_gpu 1200 python -m pytest tests -m gpu -q ;;
    bench) run bench 600 python bench.py ;;
    benchq) run benchq 300 python bench.py --steps 10 --warmup 3 --no-cpu ;;
    benchpp) run benchpp 300 bash -c "python bench.py --steps 20 --warmup 3 --no-cpu --round-trip-steps 0 --per-plane && python bench.py --steps 20 --warmup 3 --no-cpu --round-trip-steps 0 && python bench.py --steps 20 --warmup 3 --no-cpu --round-trip-steps 0 --per-plane && python bench.py --steps 20 --warmup 3 --no-cpu --round-trip-steps 0" ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu --round-trip-steps 0 ;;
    pmcf) run pmcf 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --round-trip-steps 0 ;;
    pmcw) run pmcw 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --round-trip-steps 0 ;;
    pmcsq) run pmcsq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --round-trip-steps 0 ;;
    pmcsq2) run pmcsq2 600 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU -d $OUT/pmc_sq2 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --round-trip-steps 0 ;;
    rehearse2) run rehearse2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --frames 16 --no-cpu --backend gloo ;;
    list) run list 120 rocprofv3 -L ;;
    traffic) run traffic 60 bash -c "python tools/pmc_traffic.py $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_write/run_counter_collection.csv --frames 64 --kind uniform -o $OUT/traffic.json && cp $OUT/traffic.json profiles/traffic.json" ;;
    ablate) run ablate 300 python tools/ablate_bench.py ;;
    pmcv2c) run pmcv2c 600 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD -d $OUT/pmc_v2c -o run --output-format csv -- python tools/ab_bench.py --variants 2 --rounds 4 ;;
    pmcv2d) run pmcv2d 600 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum -d $OUT/pmc_v2d -o run --output-format csv -- python tools/ab_bench.py --variants 2 --rounds 4 ;;
    pmcv2) run pmcv2 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc_v2 -o run --output-format csv -- python tools/ab_bench.py --variants 2 --rounds 4 ;;
    pmcv2b) run pmcv2b 600 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -d $OUT/pmc_v2b -o run --output-format csv -- python tools/ab_bench.py --variants 2 --rounds 4 ;;
    abb) run abb 300 python tools/ab_bench.py --variants 2 --b2b 20 ;;
    ceil) run ceil 120 tools/ubench/stream_ceiling ;;
    ceil2) run ceil2 120 tools/ubench/stream_ceiling2 ;;
    ceil3) run ceil3 120 tools/ubench/stream_ceiling3 ;;
    ceil4) run ceil4 180 tools/ubench/stream_ceiling4 ;;
    mix) run mix 300 tools/ubench/hbm_mix 2 ;;
    mix2) run mix2 300 tools/ubench/hbm_mix2 10 ;;
    mix3) run mix3 300 tools/ubench/hbm_mix3 10 ;;
    mix4) run mix4 300 tools/ubench/hbm_mix4 10 ;;
    move5a) run move5a 180 tools/ubench/move5 12 3 ;;
    testnew) run pytest_new 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "stash or dist_legs or gpus2 or bench_json" ;;
    move5b) run move5b 180 tools/ubench/move5 12 3 ;;
    abg) run abg 500 python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_g12.so tools/ubench/libvar_g16.so tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so tools/ubench/libvar_g48.so movement ;;
    abgb) run abgb 500 python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_g12.so tools/ubench/libvar_g16.so tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so tools/ubench/libvar_g48.so movement ;;
    abgx) run abgx 500 bash -c "python tools/lib_ab.py --rounds 6 --b2b 3 --kind extreme --quality 10 default tools/ubench/libvar_g16.so tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so && python tools/lib_ab.py --rounds 6 --b2b 3 --kind smooth --quality 90 --adaptive 1 default tools/ubench/libvar_g16.so tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so && python tools/lib_ab.py --rounds 6 --b2b 3 --kind const default tools/ubench/libvar_g16.so tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so" ;;
    abmv) run abmv 500 python tools/lib_ab.py --rounds 10 --b2b 3 default movement movement:tools/ubench/libvar_mv8.so movement:tools/ubench/libvar_mvnotab.so movement:tools/ubench/libvar_mvb64.so movement:tools/ubench/libvar_mvb64notab.so ;;
    abmvs) run abmvs 500 python tools/lib_ab.py --rounds 10 --b2b 3 default movement movement:tools/ubench/libvar_mvs16.so movement:tools/ubench/libvar_mvs48.so movement:tools/ubench/libvar_mvs96.so ;;
    abth) run abth 600 bash -c "python tools/lib_ab.py --rounds 6 --b2b 3 --quality 100 default tools/ubench/libvar_th3.so tools/ubench/libvar_v2g16.so movement && python tools/lib_ab.py --rounds 6 --b2b 3 --quality 99 --adaptive 1 default tools/ubench/libvar_th3.so tools/ubench/libvar_v2g16.so && python tools/lib_ab.py --rounds 6 --b2b 3 --quality 97 default tools/ubench/libvar_th3.so tools/ubench/libvar_v2g16.so && python tools/lib_ab.py --rounds 6 --b2b 3 --quality 100 --kind smooth default tools/ubench/libvar_th3.so tools/ubench/libvar_v2g16.so && python tools/lib_ab.py --rounds 6 --b2b 3 --quality 100 --kind extreme default tools/ubench/libvar_th3.so tools/ubench/libvar_v2g16.so" ;;
    auxab) run auxab 400 python tools/aux_ab.py ;;
    rtab) run rtab 400 python tools/rt_bench.py 64 ;;
    abv3) run abv3 400 python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_tabov.so tools/ubench/libvar_dyn1.so tools/ubench/libvar_dyn2.so tools/ubench/libvar_grid4.so tools/ubench/libvar_grid16.so movement ;;
    abv3b) run abv3b 400 python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_tabov.so tools/ubench/libvar_dyn1.so tools/ubench/libvar_dyn2.so tools/ubench/libvar_grid4.so tools/ubench/libvar_grid16.so movement ;;
    phase) run phase 120 tools/ubench/hbm_phase 8 ;;
    planes) run planes 300 python tools/plane_bench.py ;;
    legacy) run legacy 120 host/legacy_latency ;;
    rleab) run rleab 300 python tools/rle_ab.py ;;
    hufab) run hufab 300 python tools/huf_ab.py ;;
    smallab) run smallab 300 python tools/small_ab.py ;;
    matrix) run matrix 300 python tools/perf_matrix.py ;;
    ab43) run ab43 300 bash -c "python tools/ab_bench.py --variants 4,3 --rounds 12 && python tools/ab_bench.py --variants 4,3 --rounds 8 --kind smooth && python tools/ab_bench.py --variants 4,3 --rounds 6 --kind extreme --quality 10 && python tools/ab_bench.py --variants 4,3 --rounds 6 --adaptive 1" ;;
    clk) run clk 600 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $OUT/pmc_clk -o run --output-format csv -- python tools/ablate_bench.py ;;
    aux) run aux 300 python tools/aux_bench.py ;;
    testhuf) run pytest_huf 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "huffman or rle" ;;
    enc) run enc 300 python tools/enc_bench.py ;;
    profenc) run profenc 600 rocprofv3 --kernel-trace --stats -d $OUT/profenc -o run --output-format csv -- python tools/enc_bench.py ;;
    profaux) run profaux 600 rocprofv3 --kernel-trace --stats -d $OUT/profaux -o run --output-format csv -- python tools/aux_bench.py ;;
    rtb) run rtb 300 bash -c "python tools/rt_bench.py 64 && python tools/rt_bench.py 64 --adaptive" ;;
    testrt) run pytest_rt 600 python -m pytest tests -m gpu -x -q -k "round_trip or planes" ;;
    pmcq1) run pmcq1 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_q1 -o run --output-format csv -- python tools/ab_bench.py --variants 2 --rounds 3 ;;
    pmcq2) run pmcq2 600 rocprofv3 --pmc SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS -d $OUT/pmc_q2 -o run --output-format csv -- python tools/ab_bench.py --variants 2 --rounds 3 ;;
    pmcs1) run pmcs1 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_s1 -o run --output-format csv -- tools/ubench/stream_ceiling2 ;;
    pmcs2) run pmcs2 600 rocprofv3 --pmc SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS -d $OUT/pmc_s2 -o run --output-format csv -- tools/ubench/stream_ceiling2 ;;
    pmca1) run pmca1 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_a1 -o run --output-format csv -- python tools/aux_bench.py 16 ;;
    pmca2) run pmca2 600 rocprofv3 --pmc SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS -d $OUT/pmc_a2 -o run --output-format csv -- python tools/aux_bench.py 16 ;;
    ab23) run ab23 300 bash -c "python tools/ab_bench.py --variants 2,3 --rounds 12 && python tools/ab_bench.py --variants 2,3 --rounds 8 --kind smooth && python tools/ab_bench.py --variants 2,3 --rounds 6 --kind const && python tools/ab_bench.py --variants 2,3 --rounds 6 --adaptive 1 && python tools/ab_bench.py --variants 2,3 --rounds 6 --quality 90" ;;
    ab234) run ab234 300 bash -c "python tools/ab_bench.py --variants 2,3,4 --rounds 12 && python tools/ab_bench.py --variants 2,3,4 --rounds 8 --kind smooth && python tools/ab_bench.py --variants 2,3,4 --rounds 6 --kind const" ;;
    ab) run ab 300 python tools/ab_bench.py --variants 1,2 ;;
    abk) run abk 300 bash -c "python tools/ab_bench.py --kind smooth && python tools/ab_bench.py --kind const && python tools/ab_bench.py --adaptive 1 && python tools/ab_bench.py --quality 90" ;;
    stepov) run stepov 300 python tools/step_overhead.py ;;
    abth2) run abth2 700 bash -c "python tools/lib_ab.py --rounds 6 --b2b 3 --quality 100 default tools/ubench/libvar_th3.so tools/ubench/libvar_th3g8.so tools/ubench/libvar_th3lf.so tools/ubench/libvar_th3nz.so tools/ubench/libvar_th3all.so movement && python tools/lib_ab.py --rounds 6 --b2b 3 --quality 100 --kind smooth default tools/ubench/libvar_th3g8.so tools/ubench/libvar_th3all.so && python tools/lib_ab.py --rounds 6 --b2b 3 --quality 99 --adaptive 1 default tools/ubench/libvar_th3g8.so tools/ubench/libvar_th3all.so && python tools/lib_ab.py --rounds 6 --b2b 3 --quality 97 default tools/ubench/libvar_th3g8.so tools/ubench/libvar_th3all.so" ;;
    abq50) run abq50 500 bash -c "python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_nz.so tools/ubench/libvar_lf.so movement && python tools/lib_ab.py --rounds 6 --b2b 3 --kind extreme --quality 10 default tools/ubench/libvar_nz.so tools/ubench/libvar_lf.so && python tools/lib_ab.py --rounds 6 --b2b 3 --kind smooth --quality 90 --adaptive 1 default tools/ubench/libvar_nz.so tools/ubench/libvar_lf.so" ;;
    abth3) run abth3 900 bash -c "python tools/lib_ab.py --rounds 12 --b2b 3 --quality 100 default tools/ubench/libvar_nz.so tools/ubench/libvar_th3nz.so tools/ubench/libvar_th3nzlf.so tools/ubench/libvar_th3all.so movement movement8 && python tools/lib_ab.py --rounds 12 --b2b 3 --quality 100 --kind smooth default tools/ubench/libvar_nz.so tools/ubench/libvar_th3nz.so tools/ubench/libvar_th3nzlf.so tools/ubench/libvar_th3all.so movement movement8 && python tools/lib_ab.py --rounds 12 --b2b 3 --quality 100 --kind extreme default tools/ubench/libvar_nz.so tools/ubench/libvar_th3nz.so tools/ubench/libvar_th3nzlf.so tools/ubench/libvar_th3all.so movement movement8 && python tools/lib_ab.py --rounds 12 --b2b 3 --quality 99 --adaptive 1 default tools/ubench/libvar_nz.so tools/ubench/libvar_th3nz.so tools/ubench/libvar_th3nzlf.so tools/ubench/libvar_th3all.so movement movement8 && python tools/lib_ab.py --rounds 12 --b2b 3 --quality 97 default tools/ubench/libvar_nz.so tools/ubench/libvar_th3nz.so tools/ubench/libvar_th3nzlf.so tools/ubench/libvar_th3all.so movement movement8" ;;
    abgw1) run abgw1 900 bash -c "python tools/lib_ab.py --rounds 10 --b2b 3 --quality 100 default tools/ubench/libvar_ctl.so tools/ubench/libvar_pctl.so tools/ubench/libvar_pnz.so tools/ubench/libvar_pth3.so tools/ubench/libvar_pgw.so movement8 && python tools/lib_ab.py --rounds 10 --b2b 3 --quality 100 --kind smooth default tools/ubench/libvar_ctl.so tools/ubench/libvar_pctl.so tools/ubench/libvar_pnz.so tools/ubench/libvar_pth3.so tools/ubench/libvar_pgw.so movement8 && python tools/lib_ab.py --rounds 10 --b2b 3 --quality 99 --adaptive 1 default tools/ubench/libvar_ctl.so tools/ubench/libvar_pctl.so tools/ubench/libvar_pnz.so tools/ubench/libvar_pth3.so tools/ubench/libvar_pgw.so movement8" ;;
    abgw2) run abgw2 900 bash -c "python tools/lib_ab.py --rounds 10 --b2b 3 --quality 50 default tools/ubench/libvar_pctl.so tools/ubench/libvar_pnz.so tools/ubench/libvar_pgw.so movement8 && python tools/lib_ab.py --rounds 10 --b2b 3 --quality 10 --kind extreme default tools/ubench/libvar_pctl.so tools/ubench/libvar_pnz.so tools/ubench/libvar_pgw.so movement8 && python tools/lib_ab.py --rounds 10 --b2b 3 --quality 97 default tools/ubench/libvar_pctl.so tools/ubench/libvar_pnz.so tools/ubench/libvar_pgw.so movement8" ;;
    rtgw) run rtgw 400 bash -c "python tools/rt_bench.py 64 && python tools/rt_bench.py 64 --kind=extreme --q=10" ;;
    hpgw) run hpgw 400 bash -c "python tools/huf_pixels_ab.py uniform 50 && python tools/huf_pixels_ab.py extreme 10" ;;
    order) run order 900 bash -c "python tools/lib_ab.py --rounds 10 --b2b 3 --quality 100 tools/ubench/libvar_pctl.so default tools/ubench/libvar_copy.so tools/ubench/libvar_pnz.so && python tools/lib_ab.py --rounds 10 --b2b 3 --quality 100 tools/ubench/libvar_copy.so tools/ubench/libvar_pctl.so default && python tools/lib_ab.py --rounds 10 --b2b 3 --quality 100 default tools/ubench/libvar_copy.so tools/ubench/libvar_pctl.so && python tools/lib_ab.py --rounds 10 --b2b 3 --quality 50 tools/ubench/libvar_copy.so default tools/ubench/libvar_pctl.so" ;;
    hpw) run hpw 500 bash -c "python tools/huf_pixels_ab.py uniform 50 && python tools/huf_pixels_ab.py extreme 10 && python tools/huf_pixels_ab.py smooth 90 && python tools/huf_pixels_ab.py uniform 99" ;;
    abnz) run abnz 500 bash -c "python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_nz0.so movement8 && python tools/lib_ab.py --rounds 8 --b2b 3 --quality 100 default tools/ubench/libvar_nz0.so movement8 && python tools/lib_ab.py --rounds 8 --b2b 3 --kind extreme --quality 10 default tools/ubench/libvar_nz0.so" ;;
    abwt) run abwt 900 bash -c "python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_wt.so tools/ubench/libvar_wt24.so tools/ubench/libvar_wt32.so tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so movement movement8 movement:tools/ubench/libvar_mwt.so movement:tools/ubench/libvar_mwt32.so && python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_wt.so tools/ubench/libvar_wt24.so tools/ubench/libvar_wt32.so tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so movement movement8 movement:tools/ubench/libvar_mwt.so movement:tools/ubench/libvar_mwt32.so && python tools/lib_ab.py --rounds 8 --b2b 3 --kind extreme --quality 10 default tools/ubench/libvar_wt.so tools/ubench/libvar_wt24.so tools/ubench/libvar_wt32.so tools/ubench/libvar_g24.so && python tools/lib_ab.py --rounds 8 --b2b 3 --kind smooth --quality 90 --adaptive 1 default tools/ubench/libvar_wt.so tools/ubench/libvar_wt24.so tools/ubench/libvar_wt32.so tools/ubench/libvar_g24.so" ;;
    move6) run move6 300 tools/ubench/move6 12 3 ;;
    move7) run move7 300 tools/ubench/move7 12 3 ;;
    move8) run move8 300 tools/ubench/move8 12 3 ;;
    abpin) run abpin 900 bash -c "python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_pin.so movement movement:tools/ubench/libvar_mpin.so movement8 && python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_pin.so movement movement:tools/ubench/libvar_mpin.so movement8 && python tools/lib_ab.py --rounds 8 --b2b 3 --kind extreme --quality 10 default tools/ubench/libvar_pin.so && python tools/lib_ab.py --rounds 8 --b2b 3 --kind smooth --quality 90 --adaptive 1 default tools/ubench/libvar_pin.so" ;;
    abfo) run abfo 900 bash -c "python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_prev.so tools/ubench/libvar_pin0.so tools/ubench/libvar_g32.so movement movement8 && python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_prev.so tools/ubench/libvar_pin0.so tools/ubench/libvar_g32.so movement movement8 && python tools/lib_ab.py --rounds 8 --b2b 3 --kind extreme --quality 10 default tools/ubench/libvar_prev.so tools/ubench/libvar_g32.so && python tools/lib_ab.py --rounds 8 --b2b 3 --kind smooth --quality 90 --adaptive 1 default tools/ubench/libvar_prev.so tools/ubench/libvar_g32.so && python tools/lib_ab.py --rounds 8 --b2b 3 --quality 100 default tools/ubench/libvar_prev.so tools/ubench/libvar_g32.so movement8" ;;
    abgrid) run abgrid 900 bash -c "python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so tools/ubench/libvar_g48.so movement movement8 && python tools/lib_ab.py --rounds 10 --b2b 3 default tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so tools/ubench/libvar_g48.so movement movement8 && python tools/lib_ab.py --rounds 8 --b2b 3 --kind extreme --quality 10 default tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so tools/ubench/libvar_g48.so && python tools/lib_ab.py --rounds 8 --b2b 3 --kind smooth --quality 90 --adaptive 1 default tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so tools/ubench/libvar_g48.so && python tools/lib_ab.py --rounds 8 --b2b 3 --kind const default tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so tools/ubench/libvar_g48.so && python tools/lib_ab.py --rounds 8 --b2b 3 --frames 4 default tools/ubench/libvar_g24.so tools/ubench/libvar_g32.so tools/ubench/libvar_g48.so" ;;
    abv2g) run abv2g 900 bash -c "python tools/lib_ab.py --rounds 8 --b2b 3 --quality 100 default tools/ubench/libvar_ctl.so tools/ubench/libvar_v2gw.so movement8 && python tools/lib_ab.py --rounds 8 --b2b 3 --quality 100 --kind smooth default tools/ubench/libvar_ctl.so tools/ubench/libvar_v2gw.so movement8 && python tools/lib_ab.py --rounds 8 --b2b 3 --quality 99 --adaptive 1 default tools/ubench/libvar_ctl.so tools/ubench/libvar_v2gw.so movement8 && python tools/lib_ab.py --rounds 8 --b2b 3 --quality 99 default tools/ubench/libvar_ctl.so tools/ubench/libvar_v2gw.so movement8 && python tools/lib_ab.py --rounds 8 --b2b 3 --quality 97 default tools/ubench/libvar_ctl.so tools/ubench/libvar_v2gw.so movement8 && python tools/lib_ab.py --rounds 8 --b2b 3 --quality 100 --kind extreme default tools/ubench/libvar_ctl.so tools/ubench/libvar_v2gw.so movement8" ;;
    collect) run collect 1100 bash tools/collect_profiles.sh ;;
    probe) run probe 400 bash -c "python tools/lib_order_probe.py product && python tools/lib_order_probe.py diag && python tools/lib_order_probe.py both && python tools/lib_order_probe.py streams && python tools/lib_order_probe.py both 50 && python tools/lib_order_probe.py diag && python tools/lib_order_probe.py product" ;;
    testdist) run pytest_dist 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "gpus2 or dist_legs or bench_json" ;;
    matrix2) run matrix2 400 python tools/perf_matrix.py ;;
    aux2) run aux2 300 python tools/aux_bench.py ;;
    profaux2) run profaux2 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profaux2 -o run --output-format csv -- python tools/aux_bench.py ;;
    huf2) run huf2 300 python tools/huf_ab.py ;;
    rehearse8) run rehearse8 600 python bench.py --gpus 8 --backend gloo --frames 4 --total-frames 8 --no-cpu --ceiling-rounds 2 --steps 5 --warmup 2 --encode-steps 3 --round-trip-steps 3 --gather-steps 2 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session done"
