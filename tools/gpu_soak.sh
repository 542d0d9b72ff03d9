# Soak: 2000 config-4 steps (8.2 M frames) fp32 and fp16 storage; bench exits non-zero on any hand-off timeout
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/soak; mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 3 --no-extras --cpu-seconds 0 --no-check > $O/f32.log 2>&1; rc=$?
echo "fp32 rc=$rc"; grep -h '^{' $O/f32.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; [ $rc -ne 0 ] && { tail -5 $O/f32.log; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 3 --no-extras --cpu-seconds 0 --no-check --fp16 > $O/f16.log 2>&1; rc=$?
echo "fp16 rc=$rc"; grep -h '^{' $O/f16.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; exit $rc
