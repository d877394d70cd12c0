# Phase timing of the M32768 x N1024 x K512 BN-backward dgrad with and without the epilogue token
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r6t}
for v in ts_notok ts_tok ts_notok ts_tok; do
  echo "== $v"
  URED_LIB=$GRAFT_REPO_ROOT/build_ab/$v.so timeout -k 10 300 python tools/gemm_phase.py 2>/dev/null | grep -v '^{' || exit 1
done > gpurun_out/${TAG}_token_phase.log
cat gpurun_out/${TAG}_token_phase.log
