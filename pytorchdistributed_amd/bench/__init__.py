"""Benchmarks: ResNet-50 DDP scaling (headline), NB03 model/pipeline-parallel parity and the
split-size sweep, GPT-2 DDP, Llama-3 FSDP, GPT-2-XL PPxDP, collective micro-benchmarks."""
