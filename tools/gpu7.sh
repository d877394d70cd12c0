set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/t_all.log 2>&1
echo "pytest rc=$?" >> gpurun_out/t_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke rc=$?" >> gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r1 -o step --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-breakdown > $R/gpurun_out/prof_r1.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_fetch -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown > $R/gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pmc_write -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown > $R/gpurun_out/pmc_write.log 2>&1
echo "prof rc=$?" >> $R/gpurun_out/prof_r1.log
