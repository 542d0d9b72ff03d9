# A/B of library builds under ab/ (tools/ab_build.sh): [MODE=onepass|xcd] tools/gpu_ab.sh "name1 name2 ..." [F] [reps] [rounds]
cd $GRAFT_REPO_ROOT
names=$1; F=${2:-4096}; R=${3:-20}; N=${4:-2}
for i in $(seq $N); do
  for n in $names; do
    echo -n "$n: "
    FMCW_LIB=ab/$n.so timeout -k 10 120 python -u tools/onepass_perf.py $F $R ${MODE:-onepass} > gpurun_out/ab_$n.log 2>&1 || { tail -5 gpurun_out/ab_$n.log; exit 1; }
    grep -E "^onepass|^xcd|k_rd1p|xk-stamps| onepass " gpurun_out/ab_$n.log | tr -s ' ' | tr '\n' ' '; echo
  done
done
