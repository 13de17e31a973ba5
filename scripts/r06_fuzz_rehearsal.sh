# round 6: a long fuzz of the AUTO policy on the final library (a fresh seed
# range), then the bare two-rank rehearsal with the final bench.py
set -o pipefail
TCPCK_FUZZ_BASE=600000 TCPCK_FUZZ_SEEDS=1500 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py > gpurun_out/r06_fuzz_long.log 2>&1 &&
TCPCK_BENCH_BACKEND=gloo TCPCK_BENCH_DEVICE=0 timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/r06_bare_gpus2_rehearsal_final.json 2> gpurun_out/r06_bare_gpus2_rehearsal_final.err
