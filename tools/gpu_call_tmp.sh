set -o pipefail
mkdir -p gpurun_out/p2
timeout -k 5 120 python tools/probe/run_vq_probe.py 4 8 > gpurun_out/p2/vqprobe.txt 2>&1; cat gpurun_out/p2/vqprobe.txt | grep wpc
bash tools/gpu_check.sh r01_s2b
