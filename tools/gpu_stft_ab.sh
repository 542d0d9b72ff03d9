# STFT leg timing (tools/stft_perf.py) at several persistent-grid sizes, kernel stats, and one
# bench line.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { n=$1; shift; timeout -k 10 120 "$@" > gpurun_out/sp_$n.log 2>&1; rc=$?; echo "== $n rc=$rc"; grep -E "us per call|L =" gpurun_out/sp_$n.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/sp_$n.log; exit $rc; }; }
run base python -u tools/stft_perf.py 50
for b in ${BPCS:-2 4 6}; do run bpc$b env FMCW_STFT64_BPC=$b python -u tools/stft_perf.py 50 max,direct,stored; done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sp_stats -o run --output-format csv -- python3 tools/stft_perf.py 20 > gpurun_out/sp_stats.log 2>&1; echo "stats rc=$?"
