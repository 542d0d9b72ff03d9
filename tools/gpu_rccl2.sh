set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 90 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/rccl_samedev.py > gpurun_out/rccl2.log 2>&1; rc=$?
echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/rccl2.log | tail -12
