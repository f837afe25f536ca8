"""Autograd-aware operators over the CDNA4 HIP kernels.

Layout conventions: convolution activations are channels-last ``[N, H, W, C]`` tensors, convolution
weights are ``[C_out, R, S, C_in]`` (OHWI).  Every op has exactly one GPU implementation (the native
kernel, which raises if the extension is missing) and a PyTorch reference implementation used for
CPU tensors (tests, the gloo plumbing config) and as the numerics oracle.
"""
from .conv import conv2d, conv2d_bn_stats  # noqa: F401
from .linear import linear, mlp_gelu  # noqa: F401
from .quant import Int8Linear, quantize_int8, quantize_linears, w8_linear  # noqa: F401
from .norm import add_norm, add_norm_train, batch_norm, batch_norm_dual, dual_bn_ok, layer_norm, rms_norm  # noqa: F401
from .pool import bn_relu_max_pool2d, max_pool2d, global_avg_pool2d  # noqa: F401
from .loss import cross_entropy  # noqa: F401
from .act import relu, gelu_tanh, swiglu  # noqa: F401
from .synth import fill_normal_, fill_uniform_, fill_randint_  # noqa: F401
from .attention import (attention_cached, attention_qkv, attention_ref, decode_attention, embedding,  # noqa: F401
                        rope_tables)
