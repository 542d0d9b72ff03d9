# Per-phase step times of k_rdx (ab/stamps.so, -DXK_STAMPS), fp32 and fp16 storage
set -u
cd $GRAFT_REPO_ROOT
for f in 0 1; do
  FP16=$f FMCW_LIB=ab/stamps.so timeout -k 10 120 python -u tools/onepass_perf.py 4096 2 xcd > gpurun_out/st2_$f.log 2>&1 || { echo "fp16=$f failed"; tail -5 gpurun_out/st2_$f.log; exit 1; }
  echo "fp16=$f"; grep -h "xk-stamps\|xcd" gpurun_out/st2_$f.log | tail -4
done
