"""hipBLASLt (torch.mm) vs the native MFMA GEMM (auto path and forced 256x256 wide tile) on the
GPT-2-medium training GEMMs (32 x 1024 tokens per GPU): forward, dgrad and wgrad layouts of the
qkv / proj / fc1 / fc2 projections.  Decides whether a fused-epilogue native GEMM (bias + GELU, GELU
backward) can replace the library call plus a separate elementwise pass.

    python tools/bench_gpt2_gemm.py [tokens] > out.jsonl
"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pytorchdistributed_amd._native import C  # noqa: E402


def t(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 32 * 1024
    d, f = 1024, 4096
    for name, N, K in [("qkv", 3 * d, d), ("proj", d, d), ("fc1", f, d), ("fc2", d, f)]:
        x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
        dy = torch.randn(T, N, device="cuda").to(torch.bfloat16)
        y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
        dx = torch.empty(T, K, device="cuda", dtype=torch.bfloat16)
        dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        cases = {
            # forward y = x W^T
            "fwd": (lambda: torch.mm(x, w.t(), out=y),
                    lambda: C().gemm(x, True, K, w, True, K, y, N, T, N, K, None, False, True)),
            # dgrad dx = dy W
            "dgrad": (lambda: torch.mm(dy, w, out=dx),
                      lambda: C().gemm(dy, True, N, w, False, K, dx, K, T, K, N, None, False, True)),
            # wgrad dw = dy^T x
            "wgrad": (lambda: torch.mm(dy.t(), x, out=dw),
                      lambda: C().gemm(dy, False, N, x, False, K, dw, K, N, K, T, None, False, True)),
        }
        fl = 2 * T * N * K
        for kind, (blas, native) in cases.items():
            tb = t(blas)
            C().set_gemm_paths(-1)
            ta = t(native)
            C().set_gemm_paths(2)
            tw = t(native)
            C().set_gemm_paths(-1)
            print(json.dumps({"gemm": name, "kind": kind, "M": T, "N": N, "K": K,
                              "blas_ms": round(tb, 4), "blas_tflops": round(fl / tb / 1e9, 1),
                              "native_auto_ms": round(ta, 4), "native_auto_tflops": round(fl / ta / 1e9, 1),
                              "native_wide_ms": round(tw, 4), "native_wide_tflops": round(fl / tw / 1e9, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
