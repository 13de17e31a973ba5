set -e
for c in fill slots receive segment c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-e2e > gpurun_out/alone_$c.log 2>&1
done
timeout -k 10 400 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/order_default.log 2>&1
