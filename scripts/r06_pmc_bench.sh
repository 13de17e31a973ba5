# round 6: every bench key's FETCH_SIZE / WRITE_SIZE pass on the final library,
# the summary (profiles/pmc_summary.json, stamped with the library's sha256),
# then the driver's default bench command reading it
set -o pipefail
STEPS="pmc_all" bash scripts/gpu_check.sh > gpurun_out/r06_pmc_all.log 2>&1 &&
python3 scripts/pmc_summary.py r06 > gpurun_out/r06_pmc_summary.log 2>&1 &&
cp profiles/pmc_summary.json gpurun_out/pmc_summary_r06.json &&
timeout -k 10 600 python bench.py > gpurun_out/r06_bench_final.json 2> gpurun_out/r06_bench_final.err
