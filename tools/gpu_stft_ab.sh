# STFT leg diagnostics (tools/stft_perf.py under the FMCW_STFT64_* knobs), PMC of the nfft-64
# kernels, and one bench line.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { n=$1; shift; timeout -k 10 120 "$@" > gpurun_out/sp_$n.log 2>&1; rc=$?; echo "== $n rc=$rc"; grep -E "us per call|L =" gpurun_out/sp_$n.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/sp_$n.log; exit $rc; }; }
run base python -u tools/stft_perf.py 50
run nogather env FMCW_STFT64_DBG=1 python -u tools/stft_perf.py 50 max,direct,stored
run nomfma env FMCW_STFT64_DBG=2 python -u tools/stft_perf.py 50 max,direct,stored
run nostore env FMCW_STFT64_DBG=4 python -u tools/stft_perf.py 50 max,direct,stored
run none env FMCW_STFT64_DBG=7 python -u tools/stft_perf.py 50 max,direct,stored
for b in 1 2 4 8; do run bpc$b env FMCW_STFT64_BPC=$b python -u tools/stft_perf.py 50 max,direct,stored; done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/sp_pmc -o run --output-format csv -- python3 tools/stft_perf.py 5 max,direct > gpurun_out/sp_pmc.log 2>&1; echo "pmc rc=$?"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sp_stats -o run --output-format csv -- python3 tools/stft_perf.py 20 > gpurun_out/sp_stats.log 2>&1; echo "stats rc=$?"
timeout -k 10 600 python -u bench.py --cpu-seconds 0 --no-host-path > gpurun_out/sp_bench.log 2>&1; echo "bench rc=$?"
