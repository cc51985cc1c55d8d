"""Dev: one packed + fused + prefill-attention LLaMA3-8B-shaped window under rocprofv3 (kernel
time breakdown of the PPL eval loop); LAYERS (default 8), WINDOWS (default 2)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from models.quant_llama import build_random_quant_llama, quant_args, rtn_quantize_
from transformers import LlamaConfig

L = int(os.environ.get("LAYERS", "8"))
W = int(os.environ.get("WINDOWS", "2"))
cfg = LlamaConfig(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                  num_key_value_heads=8, num_hidden_layers=L, vocab_size=128256,
                  max_position_embeddings=8192, rms_norm_eps=1e-5, rope_theta=500000.0)
dev = torch.device("cuda:0")
model = build_random_quant_llama(cfg, quant_args(4, 128), seed=3, device=dev, dtype=torch.float16)
rtn_quantize_(model, pack=True)
for layer in model.layers:
    layer.fuse_packed_projections(prefill_attention=True)
g = torch.Generator(device=dev).manual_seed(1)
toks = torch.randint(0, cfg.vocab_size, (1, W * 2048), device=dev, generator=g)
with torch.no_grad():
    for i in range(W):
        logits = model(toks[:, i * 2048:(i + 1) * 2048])
        del logits
torch.cuda.synchronize()
print("done", flush=True)
