# Round-4 probe part L: role split, with PMC.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04l_probe
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 tools/r04_probe.bin 12 > $O/probe12_$r.log 2>&1; rc=$?
  cat $O/probe12_$r.log; [ $rc -ne 0 ] && { echo "probe rc=$rc"; exit $rc; }
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/p12_$c -o run --output-format csv -- tools/r04_probe.bin 12 > $O/p12_$c.log 2>&1 || { echo "pmc failed"; tail -3 $O/p12_$c.log; exit 1; }
done
echo call done
