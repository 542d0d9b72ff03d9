#!/bin/bash
# LDS / issue counters of k_rdx for library variants (one rocprofv3 --pmc pass each):
#   tools/pmc_lds.sh "name1 name2 ..."   (ab/<name>.so; "prod" = the in-tree library)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in $1; do
  lib=ab/$n.so; [ "$n" = prod ] && lib=fmcw_radar_processing_amd/libfmcw.so
  FMCW_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE \
    SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace -d gpurun_out/pmclds_$n -o run \
    --output-format csv -- python3 tools/onepass_perf.py 4096 2 xcd > gpurun_out/pmclds_$n.log 2>&1 || { echo "pmc $n failed"; tail -5 gpurun_out/pmclds_$n.log; exit 1; }
  python3 - gpurun_out/pmclds_$n <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)
acc = collections.defaultdict(list)
for fn in f:
    for r in csv.DictReader(open(fn)):
        if 'k_rdx' in r.get('Kernel_Name', ''):
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
print(sys.argv[1], {k: '%.4g' % (sum(v) / len(v)) for k, v in acc.items()})
PY
done
