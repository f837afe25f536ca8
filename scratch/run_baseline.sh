set -e
cd /root/repo
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))"
timeout -k 10 300 python scratch/torch_baseline.py amp_cl 256 20
timeout -k 10 300 python scratch/torch_baseline.py bf16pure_cl 256 20
timeout -k 10 300 python scratch/torch_baseline.py amp 256 20
export MIOPEN_FIND_MODE=FAST
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof_base -o prof --output-format csv -- python /root/repo/scratch/torch_baseline.py bf16pure_cl 256 10
