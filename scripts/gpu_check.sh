#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a fault/abort/timeout ends the session.
# A plain test failure (exit 1) does not stop the later steps.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
if [[ " ${STEPS:-} " == *" pmc_all "* ]]; then  # every bench key's two PMC passes, in bench order
  STEPS="${STEPS/pmc_all/pmc_c2 pmc_c5 pmc_fill pmc_fill_noout pmc_c2_rfc pmc_slots pmc_receive pmc_segment pmc_c3 pmc_fill_c3 pmc_c4}"
fi
for s in ${STEPS:-tests smoke bench prof}; do
  case $s in
    tests) step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    bench_c3) step bench_c3 600 python bench.py --config c3 --no-cpu-baseline ;;
    sweep) step sweep 900 python scripts/sweep.py ;;
    sweep_c3) step sweep_c3 600 python scripts/sweep.py --configs c3 ;;
    rv) step rv 900 python -m pytest tests/test_gpu_kernels.py -x -q -k rstream ;;
    sweep_c2) step sweep_c2 600 python scripts/sweep.py --configs c2 ;;
    diagstream) step diagstream 600 python scripts/diag_stream.py ;;
    policy) step policy 900 python scripts/policy_sweep.py ;;
    policy_fixed) step policy_fixed 900 python scripts/policy_sweep.py --no-mixes ;;
    policy_small) step policy_small 900 python scripts/policy_sweep.py --no-mixes --lengths 32,64,96,192,256,512,768,1024 --reps 4 ;;
    policy_mix) step policy_mix 900 python scripts/policy_sweep.py --no-fixed ;;
    vv) step vv 900 python -m pytest tests/test_gpu_kernels.py -x -q -k vvstream ;;
    bench_c4) step bench_c4 600 python bench.py --config c4 --no-cpu-baseline ;;
    bench_c5) step bench_c5 600 python bench.py --config c5 --no-cpu-baseline --no-e2e ;;
    mrank) step mrank 600 env TCPCK_BENCH_BACKEND=gloo TCPCK_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 5 --warmup 2 &&
      step mrank_c5 600 env TCPCK_BENCH_BACKEND=gloo TCPCK_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 2 --config c5 --steps 5 --warmup 2 ;;
    vvprobe) step vvprobe 600 python scripts/vv_probe.py ;;
    vvtests) step vvtests 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k vvstream ;;
    b2b_c3) step b2b_c3 600 python scripts/b2b_probe.py --what c3 ;;
    b2b_c2) step b2b_c2 600 python scripts/b2b_probe.py --what c2 ;;
    xcd_c2) step xcd_c2 600 python scripts/b2b_probe.py --what c2 --params 524298,524302,2097162,2097166,2097167,1048586,1048590 ;;
    tr_c3) step tr_c3 300 python scripts/transient.py --what c3 ;;
    tr_c2) step tr_c2 300 python scripts/transient.py --what c2 --n 800 ;;
    fillprobe) step fillprobe 600 python scripts/fill_probe.py ;;
    vvall) step vvall 900 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k vvstream ;;
    fillwrite) step fillwrite 300 python scripts/fill_write_probe.py ;;
    cpol) step cpol 300 python scripts/cpol_probe.py ;;
    os_c4) step os_c4 600 python scripts/oversub.py --what c4,c4r,c4v --ms 1,2,4,8,16,32 ;;
    gap) step gap 600 python scripts/gap_probe.py ;;
    os_c5) step os_c5 600 python scripts/oversub.py --what c5,c5v,c2v --variants 0,1,10 --ms 8,16,32,64 ;;
    xcd) step xcd_c2 300 python scripts/xcd_probe.py --what c2 && step xcd_c3 300 python scripts/xcd_probe.py --what c3 &&
      step xcd_c4 300 python scripts/xcd_probe.py --what c4 && step xcd_c5 300 python scripts/xcd_probe.py --what c5 ;;
    sq)  # SQ instruction-mix / stall passes over scripts/pmc_probe.py (8 SQ counters max per pass)
      timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
      step sq1 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/sq1 -o run --output-format csv -- python3 scripts/pmc_probe.py &&
      step sq2 120 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD -d gpurun_out/sq2 -o run --output-format csv -- python3 scripts/pmc_probe.py ;;
    gstests) step gstests 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k gstream ;;
    gssweep) step gssweep 600 python scripts/gstream_probe.py --ops checksum --lengths 32,64,128,256 --gs 0x80000,0x100000,0x200000,0x400000,0x80002,0x100002,0x200002,0x400002 ;;
    gspol) step gspol 600 python scripts/gstream_probe.py --ops checksum,fill --lengths 32,128,512 --gs 0,2,0x10,0x20,0x40,0x80,0x100,0x22 ;;
    gsfill) step gsfill 600 python scripts/gstream_probe.py --ops fill --lengths 32,64,128,256,512,1024 --gs 0,0x80,0x200,0x201,0x202 ;;
    gsorder) step gsorder 600 python scripts/gstream_probe.py --ops fill --lengths 32,256,512,1024 --gs 0,0x80,0x100,0x200,0x201,0x202 ;;
    gswb) step gswb_tests 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gstream_fill" &&
      step gswb 600 python scripts/gstream_probe.py --ops fill --lengths 32,64,128,256,512,1024 --gs 0x200,0x400,0x800,0xC00,0x401 ;;
    gsnp) step gsnp_tests 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gstream_np or gstream_reject or gstream_fill" &&
      step gsnp_fill 600 python scripts/gstream_probe.py --ops fill --lengths 48,96,128,144,192,240 --gs 0,0x80,0x400,0x401 &&
      step gsnp_ck 600 python scripts/gstream_probe.py --ops checksum --lengths 48,96,192,240 --gs 0,1,0x80 ;;
    fjumbo) step fjumbo 600 python scripts/fill_wb_probe.py --lengths 4096,4098,6144,8192,9000,12000,16384,24576,32768,49152,65536 ;;
    fjumbo3) step fjumbo3_tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "auto" &&
      step fjumbo3 600 python scripts/fill_wb_probe.py --ops checksum,fill --lengths 4098,5000,6144,9000,12000,16384,20000,24576,28000,40000,49152,60000,65536 ;;
    c2fill) step c2fill 600 python scripts/c2_fill_sweep.py ;;
    c3fill) step c3fill 600 python scripts/c3_fill_sweep.py ;;
    jlay) step jlay 600 python scripts/jumbo_layout_probe.py ;;
    jlayf) step jlayf 600 python scripts/jumbo_layout_probe.py --fill ;;
    fjumbo2) step fjumbo2 600 python scripts/fill_wb_probe.py --ops checksum,fill --lengths 5000,7000,9000,10000,14000,20000,28000,40000,49152,60000,65504 ;;
    keep) step keep 600 python scripts/keep_probe.py ;;
    vvkeep) step vvkeep 900 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "vvstream" ;;
    gsstage) step gsstage 600 python scripts/gstream_probe.py --ops checksum,fill --lengths 32,64,128,256,1024 --gs 0,2,0x800,0x802,0x80,0x880 ;;
    gsprobe) step gsprobe 600 python scripts/gstream_probe.py ;;
    resend) step resend_tests 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k set_ack &&
      step resend 300 python scripts/resend_probe.py ;;
    fdefer) step fdefer_tests 600 python -u -m pytest tests/test_gpu_fill_defer.py -x -q --timeout 120 --timeout-method thread &&
      step fdefer 300 python scripts/fill_defer_probe.py ;;
    fupd) step fupd_tests 600 python -u -m pytest tests/test_gpu_fill_update.py -x -q --timeout 120 --timeout-method thread &&
      step fupd 600 python scripts/fill_update_probe.py ;;
    rfused) step rfused_tests 600 python -u -m pytest tests/test_gpu_receive.py -x -q --timeout 120 --timeout-method thread &&
      step rfused 600 python scripts/receive_fused_probe.py ;;
    c3gap) step c3gap 600 python scripts/c3_gap_probe.py ;;
    multi) step multi_tests 600 python -u -m pytest tests/test_gpu_multi_ctx.py -x -q --timeout 120 --timeout-method thread &&
      step multi 300 python scripts/e2e_multi_probe.py ;;
    c4shape) step c4shape 600 python scripts/c4_shape_probe.py ;;
    recheck) step recheck 600 python scripts/slots_seg_recheck.py ;;
    copy) step copy 600 python scripts/copy_probe.py ;;
    fuzz) step fuzz_tests 600 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread ;;
    receive) step receive_tests 300 python -u -m pytest tests/test_gpu_receive.py -x -q --timeout 120 --timeout-method thread &&
      step receive 300 python scripts/receive_probe.py ;;
    fillpol) step fillpol 300 python scripts/fill_write_probe.py --store-policy ;;
    pmc_rs) step pmc_rs 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_rs -o run --output-format csv -- python3 scripts/pmc_probe.py --rs ;;
    os_c5x) step os_c5x 600 python scripts/oversub.py --what c5,c2 --variants 18,20,21 --ms 16,32,64,128 ;;
    pmc_vv) step pmc_vv 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_vv -o run --output-format csv -- python3 scripts/pmc_probe.py --vv ;;
    xcd23) step xcd_c2 300 python scripts/xcd_probe.py --what c2 && step xcd_c3 300 python scripts/xcd_probe.py --what c3 ;;
    reuse) step reuse 300 python scripts/reuse_probe.py ;;
    split) step split 300 python scripts/split_probe.py ;;
    c3big) step c3big 300 python scripts/xcd_probe.py --what c3big ;;
    segtests) step segtests 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread ;;
    c4x) step xcd_c4 300 python scripts/xcd_probe.py --what c4 ;;
    jumbo) step jumbo 600 python scripts/xcd_probe.py --what jumbo ;;
    iso) step iso 300 python scripts/xcd_probe.py --what iso ;;
    os_c3x) step os_c3x 600 python scripts/oversub.py --what c3 --variants 3,11 --ms 8,16,32,64 ;;
    xccmap) step xccmap 300 python scripts/xcc_map.py ;;
    xcdplace) step xcdplace 600 python scripts/xcd_place_probe.py ;;
    oversub) step oversub 600 python scripts/oversub.py ;;
    os_c2) step os_c2 600 python scripts/oversub.py --what c2 --variants 0,9,10 --ms 8,16,24,32,40,48 ;;
    os_c3) step os_c3 600 python scripts/oversub.py --what c3 --variants 2,3 --ms 8,16,32 ;;
    prof_c3) step prof_c3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e ;;
    prof_slots) step prof_slots 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_slots -o run --output-format csv -- python3 bench.py --config slots --steps 10 --warmup 2 --no-cpu-baseline --no-e2e ;;
    prof_segment) step prof_segment 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_segment -o run --output-format csv -- python3 bench.py --config segment --steps 10 --warmup 2 --no-cpu-baseline --no-e2e ;;
    segtests2) step segtests2 600 python -u -m pytest tests/test_gpu_segment.py tests/test_gpu_sstream.py -x -q --timeout 300 --timeout-method thread ;;
    prof_c4) step prof_c4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- python3 bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-extras ;;
    prof_all)  # the driver's default bench command (C2 + the c3 / c4 / c5_strong keys) under the kernel trace
      step prof_all 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_all -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e &&
      python3 scripts/bench_trace_summary.py gpurun_out/prof_all/run_kernel_trace.csv --last 20 --names c2,c5_strong,fill,fill_noout,c2_rfc,slots,receive,segment,c3,fill_c3,c4 > gpurun_out/prof_all_summary.txt ;;
    fdrain) step fdrain 300 rocprofv3 --kernel-trace -d gpurun_out/fdrain -o run --output-format csv -- python3 scripts/fill_drain_probe.py &&
      step fdrain_w 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/fdrain_w -o run --output-format csv -- python3 scripts/fill_drain_probe.py --phases stream,fill,patch,instream --steps 10 &&
      step fdrain_f 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/fdrain_f -o run --output-format csv -- python3 scripts/fill_drain_probe.py --phases stream,fill,patch,instream --steps 10 ;;
    fpol) step fpol 300 rocprofv3 --kernel-trace -d gpurun_out/fpol -o run --output-format csv -- python3 scripts/fill_drain_probe.py --phases stream,sp0,sp1,sp2,sp3,sp4,sp5,sp6,sp7,sp8,fill ;;
    fblind) step fblind 300 rocprofv3 --kernel-trace -d gpurun_out/fblind -o run --output-format csv -- python3 scripts/fill_drain_probe.py --phases stream,sg2_8,sg0_8,sg8_8,sg8_1,sg9_8,sg10_8,sg10_1,sg11_8,sg11_1,sg12_8,sg1_8,stream ;;
    fblock) step fblock_tests 600 python -u -m pytest tests/test_gpu_fill_defer.py -x -q --timeout 120 --timeout-method thread -k "block" &&
      step fblock 300 rocprofv3 --kernel-trace -d gpurun_out/fblock -o run --output-format csv -- python3 scripts/fill_drain_probe.py --phases stream,fill,block,blockend,sg8_8,block,blockend,fill ;;
    hwide) step hwide 300 python scripts/receive_fused_probe.py --wide &&
      step hwide_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hwide_trace -o run --output-format csv -- python3 scripts/receive_fused_probe.py --wide &&
      step hwide_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/hwide_fetch -o run --output-format csv -- python3 scripts/receive_fused_probe.py --wide ;;
    fgran) step fgran 300 rocprofv3 --kernel-trace -d gpurun_out/fgran -o run --output-format csv -- python3 scripts/fill_drain_probe.py --phases stream,sp8,sg1_8,sg1_0,sg2_8,sg2_7,sg2_0,sg3_8,sg3_0,instream26,instream,sp7,fill ;;
    fdvv) step fdvv 600 python scripts/fill_defer_vv_probe.py ;;
    fdsweep) step fdsweep 600 python scripts/fill_defer_vv_probe.py --sweep ;;
    fdvvt) step fdvvt 600 rocprofv3 --kernel-trace -d gpurun_out/fdvvt -o run --output-format csv -- python3 scripts/fill_defer_vv_probe.py ;;
    ftests) step ftests 600 python -u -m pytest tests/test_gpu_fill_defer.py tests/test_gpu_fill_update.py tests/test_gpu_kernels.py -k "fill or Fill" -x -q --timeout 300 --timeout-method thread ;;
    fmap) step fmap 300 rocprofv3 --kernel-trace -d gpurun_out/fmap -o run --output-format csv -- python3 scripts/fill_drain_probe.py --phases stream,sg2_8,sg4_8,sg5_8,sg6_8,sg7_8,fill,sg2_8 ;;
    wtprobe) step segwt 600 python scripts/segment_probe.py --params 0,64,128 --cases 1460:1504,1024:1056 &&
      step gswt 600 python scripts/gstream_probe.py --ops fill --lengths 32,64,128 --gs 0x401,0x801,0xC01 ;;
    rtests) step rtests 900 python -u -m pytest tests/test_gpu_receive.py tests/test_gpu_rfc_long.py -x -q --timeout 300 --timeout-method thread ;;
    fmall) step fmall 300 python scripts/fill_mall_probe.py &&
      step fmall_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fmall_trace -o run --output-format csv -- python3 scripts/fill_mall_probe.py ;;
    fuzzlong) step fuzzlong 900 env TCPCK_FUZZ_BASE=200000 TCPCK_FUZZ_SEEDS=1500 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread ;;
    bench_fill_noout) step bench_fill_noout 300 python bench.py --config fill_noout ;;
    copysize) step copysize 300 python scripts/copy_size_probe.py ;;
    rorder) step rorder 300 python scripts/receive_fused_probe.py --order ;;
    prof_fill_c3) step prof_fill_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fill_c3 -o run --output-format csv -- python3 bench.py --config fill_c3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e ;;
    new4) step new4 900 python -u -m pytest tests/test_gpu_full_paths.py -x -v --timeout 300 --timeout-method thread ;;
    tests_new) step tests_new 900 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_multi_ctx.py tests/test_drop_in.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    fsweep) step fsweep 900 python scripts/fill_policy_sweep.py ;;
    bench_receive) step bench_receive 600 python bench.py --config receive ;;
    bench_fill) step bench_fill 600 python bench.py --config fill ;;
    bench_slots) step bench_slots 600 python bench.py --config slots ;;
    bench_segment) step bench_segment 600 python bench.py --config segment ;;
    prof_fill) step prof_fill 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fill -o run --output-format csv -- python3 bench.py --config fill --steps 10 --warmup 2 --no-cpu-baseline --no-e2e ;;
    prof_receive) step prof_receive 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_receive -o run --output-format csv -- python3 bench.py --config receive --steps 10 --warmup 2 --no-cpu-baseline --no-e2e ;;
    pmc_c2|pmc_c3|pmc_c4|pmc_c5|pmc_slots|pmc_segment|pmc_receive|pmc_fill|pmc_fill_noout|pmc_fill_c3|pmc_c2_rfc)
      # separate FETCH_SIZE / WRITE_SIZE passes (TCC slots), kernel trace only; the library's sha256 beside each
      c=${s#pmc_}
      sha256sum tcp-stack_amd/libtcpck.so > gpurun_out/pmc_${c}_fetch_lib.sha256
      step ${s}_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_${c}_fetch -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-e2e --no-extras
      sha256sum tcp-stack_amd/libtcpck.so > gpurun_out/pmc_${c}_write_lib.sha256
      step ${s}_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_${c}_write -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-e2e --no-extras ;;
  esac
done
