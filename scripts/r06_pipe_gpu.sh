set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rfc_published.py > gpurun_out/r06_rfc_published.log 2>&1 &&
timeout -k 10 300 python -u scripts/fill_pipe_probe.py --ks 0,2,8,258,264 --prio 0 --only c3,c2 > gpurun_out/r06_fill_pipe_attr.log 2>&1 &&
for K in 0 2 8; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pipe_pmc_${K}_fetch -o run --output-format csv -- python3 scripts/fill_pipe_probe.py --ks $K --prio 0 --only c3 --pmc-calls 3 > gpurun_out/pipe_pmc_${K}_fetch.log 2>&1 &&
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pipe_pmc_${K}_write -o run --output-format csv -- python3 scripts/fill_pipe_probe.py --ks $K --prio 0 --only c3 --pmc-calls 3 > gpurun_out/pipe_pmc_${K}_write.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 580 --timeout-method thread tests/test_abi_asan.py > gpurun_out/r06_abi_asan.log 2>&1
