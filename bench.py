"""Driver contract entry point: `python bench.py --gpus N --steps K --warmup W`.

Runs the headline benchmark (ResNet-50 DDP images/sec, BASELINE.json config 2) on N GPUs of one node;
for N > 1 launch under `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`.
Rank 0 prints one JSON line.  See pytorchdistributed_amd/bench/resnet_ddp.py.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# (importing the package first raises GPU_MAX_HW_QUEUES before HIP initialises: see
# pytorchdistributed_amd/__init__.py:_ensure_hw_queues)
import pytorchdistributed_amd  # noqa: E402,F401
from pytorchdistributed_amd.bench.resnet_ddp import main  # noqa: E402

if __name__ == "__main__":
    main()
