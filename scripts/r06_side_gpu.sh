# round 6: the ASan host test on the device, the side-buffer FILL probe
# (parity first, then timing), then the bare two-rank rehearsals of bench.py
set -o pipefail
timeout -k 10 700 python -u -m pytest -x -v -m gpu --timeout 650 --timeout-method thread tests/test_abi_asan.py > gpurun_out/r06_abi_asan_gpu.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fill_side.py > gpurun_out/r06_fill_side_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/fill_side_probe.py > gpurun_out/r06_fill_side_probe.log 2>&1 &&
TCPCK_BENCH_BACKEND=gloo TCPCK_BENCH_DEVICE=0 timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/r06_bare_gpus2_rehearsal.json 2> gpurun_out/r06_bare_gpus2_rehearsal.err &&
{ TCPCK_BENCH_BACKEND=gloo timeout -k 10 200 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/r06_bare_gpus2_nodevice.json 2> gpurun_out/r06_bare_gpus2_nodevice.err; echo "rc=$?" >> gpurun_out/r06_bare_gpus2_nodevice.err; }
