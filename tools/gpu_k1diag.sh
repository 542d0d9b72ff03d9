# K1 diagnostic A/B: ab/k1base (shipped), ab/k1nofft (FFT skipped: data movement only, wrong
# results), ab/k1pf (round-3 prefetch form); tools/k1_perf.py alternating.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/k1diag
mkdir -p $O
for i in 1 2 3; do
  for n in k1base k1nofft k1pf; do
    echo -n "$n: "
    FMCW_LIB=ab/$n.so timeout -k 10 120 python -u tools/k1_perf.py 4096 50 > $O/k1_$n.$i.log 2>&1 || { tail -5 $O/k1_$n.$i.log; exit 1; }
    grep "^k1" $O/k1_$n.$i.log
  done
done
echo call done
