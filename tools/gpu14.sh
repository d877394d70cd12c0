# rocprofv3 kernel stats + separate FETCH_SIZE / WRITE_SIZE passes of the bench, summarised per kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_k -o k --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_k.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_f -o f --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown > $R/gpurun_out/pmc_f.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_w -o w --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown > $R/gpurun_out/pmc_w.log 2>&1 && \
cd $R && python3 tools/pmc_summary.py gpurun_out/prof_k gpurun_out/pmc_f gpurun_out/pmc_w gpurun_out/pmc_summary.json > gpurun_out/pmc_summary.log 2>&1
echo "rc=$?" >> $R/gpurun_out/pmc_summary.log
