"""Driver contract entry point: `python bench.py --gpus N --steps K --warmup W`.

Runs the headline benchmark (ResNet-50 DDP images/sec, BASELINE.json config 2) on N GPUs of one node;
for N > 1 either launch under `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`
or run `bench.py --gpus N` directly: without a launcher it starts the N ranks itself
(pytorchdistributed_amd/bench/common.py:launch_ranks).
Rank 0 prints one JSON line.  See pytorchdistributed_amd/bench/resnet_ddp.py.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# 8 hardware queues for the compute, weight-gradient and RCCL streams (a one-rank RCCL group ran 5 %
# slower at HIP's default 4: profiles/r2_hw_queues.jsonl q4 / q8); importing the package applies it
# before HIP initialises (pytorchdistributed_amd/__init__.py:_ensure_hw_queues)
os.environ.setdefault("PDA_HW_QUEUES", "8")
import pytorchdistributed_amd  # noqa: E402,F401
from pytorchdistributed_amd.bench.resnet_ddp import main  # noqa: E402

if __name__ == "__main__":
    main()
