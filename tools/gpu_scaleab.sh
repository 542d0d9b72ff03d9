set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/scaleab
FMCW_LIB=ab/before.so timeout -k 10 120 python -u tools/ab_bitwise.py save gpurun_out/scaleab/before.npz 2>&1 | grep -v amdgpu.ids | tail -1
timeout -k 10 120 python -u tools/ab_bitwise.py check gpurun_out/scaleab/before.npz 2>&1 | grep -v amdgpu.ids | tail -1; rc=$?
B="python -u bench.py --cpu-seconds 0 --no-check --no-host-path --steps 20"
for i in 1 2 3; do
  for v in before new; do
    if [ $v = before ]; then L=ab/before.so; else L=fmcw_radar_processing_amd/libfmcw.so; fi
    FMCW_LIB=$L timeout -k 10 200 $B > gpurun_out/scaleab/$v.$i.log 2>&1 || { echo "bench $v failed"; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/scaleab/$v.$i.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$v', d['value'], d['roofline']['avg_launch_us'], 'fp16', d['fp16_storage']['roofline']['avg_launch_us'], d['fp16_storage']['value'])"
  done
done
