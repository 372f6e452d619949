cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04/diag
for L in tools/exp/libtkv_amq_C0FIX.so tools/exp/libtkv_amq_C0ZERO.so main; do
  if [ $L = main ]; then unset TKV_AMQ_LIB; else export TKV_AMQ_LIB=$L; fi
  echo "## $L"
  timeout -k 10 120 python -u tools/diag_vqf_blocks.py 16384 12 32704 2>&1 | grep -v amdgpu.ids | head -30 || exit 3
done
