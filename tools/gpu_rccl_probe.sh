set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 150 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 tools/rccl_same_gpu_probe.py > gpurun_out/rccl_probe.txt 2>&1
echo "rc=$?" >> gpurun_out/rccl_probe.txt
