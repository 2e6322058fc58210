set -o pipefail
mkdir -p gpurun_out/r3c
python -c "import torch; p=torch.cuda.get_device_properties(0); print({k: getattr(p,k) for k in dir(p) if 'shared' in k or 'multi_processor' in k})"
bash tools/gpu_r3tests.sh tests/test_gpu_trainer.py tests/test_gpu_hmm.py tests/test_gpu_head.py tests/test_gpu_model.py::test_cfg2_full_size_vs_oracle tests/test_gpu_model.py::test_strong_scaling_shards_vs_oracle tests/test_gpu_configs.py || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r3c/bench.json 2> gpurun_out/r3c/bench.err || { tail -20 gpurun_out/r3c/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r3c/bench.json')); print(d['ms_per_step'], d['value']); print(json.dumps(d['cpu_baseline'], indent=1))"
