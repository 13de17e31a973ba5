# round 6: the device identity bench.py gathers (PCI address + UUID + HIP bus id), then
# the bare two-rank rehearsal and a one-GPU run with the final bench.py
set -o pipefail
timeout -k 10 120 python -c "
import sys; sys.path[:0] = ['.', 'tcp-stack_amd']
import torch, tcpck, bench
torch.cuda.init(); tcpck.Context(0).close()
p = torch.cuda.get_device_properties(0)
print('uuid', repr(str(p.uuid)), 'pci', p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
print('hip bus id', repr(bench.hip_pci_bus_id(0)), 'identity', bench.device_identity(0))
" > gpurun_out/r06_identity.log 2>&1 &&
TCPCK_BENCH_BACKEND=gloo TCPCK_BENCH_DEVICE=0 timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/r06_bare_gpus2_rehearsal_id.json 2> gpurun_out/r06_bare_gpus2_rehearsal_id.err &&
timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline > gpurun_out/r06_bench_n1_id.json 2> gpurun_out/r06_bench_n1_id.err
