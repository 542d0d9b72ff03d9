# memory-hierarchy probes (development only): MALL ring, MALL hot/cold, L2 re-read, HBM copy shapes
cd $GRAFT_REPO_ROOT
for p in mall_chain mall_probe l2_probe bw_probe; do
  echo "== $p"; timeout -k 10 150 tools/$p > gpurun_out/probe_$p.log 2>&1; rc=$?
  cat gpurun_out/probe_$p.log | tail -60
  if [ $rc -ne 0 ]; then echo "STOP $p rc=$rc"; exit $rc; fi
done
