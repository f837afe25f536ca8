"""hipBLASLt (torch.mm) vs the native GEMMs on the transformer training GEMMs: forward, dgrad and wgrad
layouts of each projection (GPT-2-medium at 32 x 1024 tokens per GPU by default; ``--model llama``
for Llama-3-8B's projections at 16 x 1024 tokens).  Native arms: the production dispatch with the
pipelined 256x256 kernel (``pp``), the same with the pipelined kernel off (the 2-stage wide tile,
``wide``), and for the weight gradient the fused dW + db entry (``wgrad_db``).  Arms interleave per
round in one process; the median round is reported.

    python tools/bench_gpt2_gemm.py [--tokens T] [--model gpt2|llama] [--kinds fwd,dgrad,wgrad] > out.jsonl
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pytorchdistributed_amd._native import C  # noqa: E402

MODELS = {
    "gpt2": [("qkv", 3072, 1024), ("proj", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096),
             ("lm_head", 50304, 1024)],
    "llama": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)],
}


def t(fn, it):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=0)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--kinds", default="fwd,dgrad,wgrad")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    T = a.tokens or (32 * 1024 if a.model == "gpt2" else 16 * 1024)
    kinds = a.kinds.split(",")
    for name, N, K in MODELS[a.model]:
        if a.only and name not in a.only.split(","):
            continue
        x = (torch.rand(T, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        dy = (torch.rand(T, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        bias = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
        dx = torch.empty(T, K, device="cuda", dtype=torch.bfloat16)
        dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        db = torch.empty(N, device="cuda", dtype=torch.bfloat16)

        def pp(on, fn):
            def run():
                C().set_gemm_pp(on)
                fn()
            return run

        cases = {
            "fwd": {"blas": lambda: torch.addmm(bias, x, w.t(), out=y),
                    "pp": pp(1, lambda: C().gemm(x, True, K, w, True, K, y, N, T, N, K, bias, False, True)),
                    "wide": pp(0, lambda: C().gemm(x, True, K, w, True, K, y, N, T, N, K, bias, False, True))},
            "dgrad": {"blas": lambda: torch.mm(dy, w, out=dx),
                      "pp": pp(1, lambda: C().gemm(dy, True, N, w, False, K, dx, K, T, K, N, None, False, True)),
                      "wide": pp(0, lambda: C().gemm(dy, True, N, w, False, K, dx, K, T, K, N, None, False, True))},
            "wgrad": {"blas": lambda: (torch.mm(dy.t(), x, out=dw), torch.sum(dy, 0, out=db)),
                      "pp": pp(1, lambda: C().gemm(dy, False, N, x, False, K, dw, K, N, K, T, None, False, True)),
                      "wgrad_db": pp(1, lambda: C().gemm_wgrad_db(dy, x, dw, db)),
                      "wide": pp(0, lambda: C().gemm(dy, False, N, x, False, K, dw, K, N, K, T, None, False, True))},
        }
        fl = 2.0 * T * N * K
        for kind in kinds:
            arms = cases[kind]
            times = {k: [] for k in arms}
            for _ in range(a.rounds):
                for k, fn in arms.items():
                    times[k].append(t(fn, a.iters))
            C().set_gemm_pp(-1)
            rec = {"gemm": name, "kind": kind, "T": T, "N": N, "K": K}
            for k, ts in times.items():
                ms = sorted(ts)[len(ts) // 2]
                rec[f"{k}_ms"] = round(ms, 4)
                rec[f"{k}_tflops"] = round(fl / ms / 1e9, 1)
            print(json.dumps(rec), flush=True)
        del x, w, dy, y, dx, dw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
