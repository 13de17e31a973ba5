# round 6, library with the AVX2 host word sum: smoke, the full GPU suite, every
# key's PMC passes (new sha256 stamps), then the default bench line reading them
set -o pipefail
STEPS="smoke tests pmc_all" bash scripts/gpu_check.sh > gpurun_out/r06_final_d.log 2>&1 &&
python3 scripts/pmc_summary.py r06 > gpurun_out/r06_pmc_summary_d.log 2>&1 &&
cp profiles/pmc_summary.json gpurun_out/pmc_summary_r06d.json &&
timeout -k 10 600 python bench.py > gpurun_out/r06_bench_final_d.json 2> gpurun_out/r06_bench_final_d.err
