# Profile set of the current tree (the bench roofline's sources): kernel trace of the timed
# replayed steps, FETCH/WRITE PMC passes, held clock and MFMA-busy passes. Usage: bash tools/profile_set.sh <tag>
set -o pipefail
T=${1:-r6a}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/prof_step.sh $T 20 > gpurun_out/${T}_prof_step.log 2>&1 || { tail -20 gpurun_out/${T}_prof_step.log; exit 1; }
head -12 gpurun_out/${T}_trace_timed_top.txt
bash tools/gpu_prof.sh $T > gpurun_out/${T}_gpu_prof.log 2>&1 || { tail -20 gpurun_out/${T}_gpu_prof.log; exit 1; }
bash tools/gpu_clock_sq.sh $T > gpurun_out/${T}_clock_sq.log 2>&1 || { tail -20 gpurun_out/${T}_clock_sq.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${T}_pmc_summary.json')); [print(k[:80], v.get('hbm_bytes_per_launch')) for k,v in [x for x in d.items() if 'gemm2' in x[0]][:8]]"
