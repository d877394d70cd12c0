# Phase timing of the M32768 x N1024 x K512 BN-backward dgrad: token / priority variants, then a
# whole-step A/B of the priority build against the token-off build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r6t2}
for v in ts_notok ts_tokp3 ts_notokp3 ts_tok; do
  echo "== $v"
  URED_LIB=$GRAFT_REPO_ROOT/build_ab/$v.so timeout -k 10 300 python tools/gemm_phase.py 2>/dev/null | grep -v '^{' | grep -E "==|epi:|K-loop|epilogue|whole tile|start->|span" || exit 1
done > gpurun_out/${TAG}_token_phase.log
cat gpurun_out/${TAG}_token_phase.log
cp build_ab/tokp3.so build_ab/ab_a.so
for rep in 1 2 3; do
  for L in tok_off tokp3; do
    r=$(URED_LIB=$GRAFT_REPO_ROOT/build_ab/$L.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-all-slots-rate --no-k16-rate --no-extras --no-loader-rate --steps 30 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); v=d['gemm_variants']; print(d['value'], 'gemm_ms', d['gemm_all']['ms_per_step'], 'dgrad', v['gemm2_kernel<false, true, 0, 0, 2, 2, 2>']['ms'], 'fwd', v['gemm2_kernel<false, false, 1, 0, 1, 2, 2>']['ms'], 'wgrad', v['gemm2_kernel<true, true, 0, 1, 3, 2, 2>']['ms'])") || exit 1
    echo "rep $rep $L $r"
  done
done | tee gpurun_out/${TAG}_step_ab.log
