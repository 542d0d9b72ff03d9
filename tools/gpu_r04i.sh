# Round-4 probe: the hand-off ring's memory type (coarse / fine-grained / uncached), with PMC.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
for a in 0 1 3; do
  CUBE_ALLOC=$a timeout -k 10 120 tools/r04_probe.bin 7 > $O/probe7_$a.log 2>&1; rc=$?
  cat $O/probe7_$a.log; [ $rc -ne 0 ] && { echo "probe rc=$rc"; exit $rc; }
done
for a in 0 3; do
  for c in FETCH_SIZE WRITE_SIZE; do
    CUBE_ALLOC=$a timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/p7_${a}_$c -o run --output-format csv -- tools/r04_probe.bin 7 > $O/p7_${a}_$c.log 2>&1 || { echo "pmc failed"; tail -3 $O/p7_${a}_$c.log; exit 1; }
  done
done
echo call done
