#!/bin/bash
# The one GPU-session script: run the named evidence steps in order, each under its own time limit,
# stopping at the first crash / timeout.  Logs and profiler output land under OUT (gpurun_out/...).
#
#   scripts/gpu_evidence.sh OUT STEP [STEP ...]
#
# Steps:
#   tests        pytest -m gpu (whole GPU suite, one process)
#   smoke        __graft_entry__.smoke()
#   bench        default bench.py line (N = 1, BASELINE configs[1])
#   bench_audio  bench.py --audio-only (configs[3])      bench_detr  bench.py --image-feats detr (configs[4])
#   trace        rocprofv3 --kernel-trace --stats over a short bench
#   traffic      two PMC passes (FETCH_SIZE / WRITE_SIZE) + scripts/pmc_traffic.py -> OUT/gemm_traffic.json
#   attn_pmc     one PMC pass of VALU / MFMA instruction counts over the attention kernels
#   attn_bits    O / LSE / dQKV dumps of this build and of $AB_LIB, compared bit for bit
#   attn_bench   isolated attention timings of this build (and of $AB_LIB when set)
#   gemm_bench   isolated NT GEMM timings on the step's shapes (scripts/gemm_bits.py) of this build (and $AB_LIB)
#   test         pytest on $TEST (a file or node id), verbose
#   gemm_bits    GEMM output dumps of this build and of $AB_LIB, compared bit for bit
#   lib_ab       step A/B: bench.py interleaved $AB_REPS times over "default" and $AB_LIB
#   dp2          gloo 2-rank rehearsal of the N > 1 bench path on one GPU
export TMPDIR=/tmp
O=$1; shift
mkdir -p "$O"
run() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
        echo "=== [$name] rc=$rc"; tail -n 6 "$O/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gemm-timing"
for s in "$@"; do
  case $s in
    tests) run tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    smoke) run smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python bench.py ;;
    bench_audio) run bench_audio 300 python bench.py --audio-only --no-cpu-baseline ;;
    bench_detr) run bench_detr 300 python bench.py --image-feats detr --no-cpu-baseline ;;
    trace) run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
             python bench.py --steps 6 --warmup 3 --no-cpu-baseline ;;
    traffic)
      run pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run -- python $B
      run pmc_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run -- python $B
      run traffic 60 python scripts/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" --out "$O/gemm_traffic.json" ;;
    attn_pmc) run attn_pmc 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
                GRBM_GUI_ACTIVE --output-format csv -d "$O/attn_pmc" -o run -- python scripts/attn_bench.py ;;
    attn_bits)
      run attn_dump_new 120 python scripts/attn_bits.py /tmp/attn_new.npz
      run attn_dump_ab 120 env MMS2UT_LIB="$AB_LIB" python scripts/attn_bits.py /tmp/attn_ab.npz
      run attn_cmp 60 python scripts/wgrad_bits.py cmp /tmp/attn_new.npz /tmp/attn_ab.npz ;;
    attn_bench)
      run attn_bench 200 python scripts/attn_bench.py
      if [ -n "$AB_LIB" ]; then run attn_bench_ab 200 env MMS2UT_LIB="$AB_LIB" python scripts/attn_bench.py; fi ;;
    gemm_bench)
      run gemm_bench 200 python scripts/gemm_bits.py /tmp/gemm_t.npz
      if [ -n "$AB_LIB" ]; then run gemm_bench_ab 200 env MMS2UT_LIB="$AB_LIB" python scripts/gemm_bits.py /tmp/gemm_t.npz; fi ;;
    test) run "test_${TEST//[^a-zA-Z0-9_]/_}" 600 python -u -m pytest "$TEST" -x -v --timeout 120 --timeout-method thread ;;
    gemm_bits)
      run gemm_dump_new 120 python scripts/gemm_bits.py /tmp/gemm_new.npz
      run gemm_dump_ab 120 env MMS2UT_LIB="$AB_LIB" python scripts/gemm_bits.py /tmp/gemm_ab.npz
      run gemm_cmp 60 python scripts/wgrad_bits.py cmp /tmp/gemm_new.npz /tmp/gemm_ab.npz ;;
    lib_ab) run lib_ab 900 python scripts/lib_ab.py "$O/lib_ab.json" "${AB_REPS:-2}" default= ab="$AB_LIB" ;;
    dp2) run dp2 600 scripts/_dp2_rehearsal.sh "$O/dp2" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
