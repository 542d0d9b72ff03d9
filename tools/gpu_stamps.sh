# Stamp-build diagnostics: tools/gpu_stamps.sh "name1 name2 ..." -> per-phase us per block + residency
cd $GRAFT_REPO_ROOT
for n in $1; do
  FMCW_LIB=ab/$n.so timeout -k 10 120 python -u tools/onepass_perf.py 4096 3 onepass > gpurun_out/st_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/st_$n.log; exit 1; }
  echo "$n: $(grep -h "stamps:" gpurun_out/st_$n.log | tail -1)"; echo "   $(grep -h stamps-waves gpurun_out/st_$n.log | tail -1)"
done
