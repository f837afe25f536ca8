"""Serving: KV-cached autoregressive generation for the transformer models (Llama-3, GPT-2), with
budget-driven multi-GPU layer placement — the capability behind the reference's
``LlamaForCausalLM.from_pretrained(..., device_map="auto")`` inference (SURVEY §2.4 W8, P10;
`03 模型并行/03_model_parallel.ipynb` raw lines 85-89)."""
from .generate import KVCache, generate, place  # noqa: F401
from .server import BatchingEngine, create_app  # noqa: F401
