"""torch.profiler breakdown of one packed LLaMA3-8B-shaped decoder layer decode step (dev)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from models.quant_llama import quant_args, random_llama_layer, rtn_quantize_
from models.int_llama_layer import QuantLlamaDecoderLayer
from quant.utils import pack_quant_linears
from transformers import LlamaConfig
cfg = LlamaConfig(hidden_size=4096, intermediate_size=14336, num_attention_heads=32, num_key_value_heads=8,
                  num_hidden_layers=1, vocab_size=128256, max_position_embeddings=8192, rms_norm_eps=1e-5,
                  rope_theta=500000.0)
dev = torch.device("cuda:0")
layer = QuantLlamaDecoderLayer(cfg, random_llama_layer(cfg, 1, dev, torch.float16), quant_args(4, 128))
class S(torch.nn.Module):
    def __init__(s, l):
        super().__init__(); s.layers = torch.nn.ModuleList([l])
rtn_quantize_(S(layer), pack=True)
layer.fuse_packed_projections()
kv = 512
past = (torch.randn(1, 8, kv, 128, device=dev, dtype=torch.float16), torch.randn(1, 8, kv, 128, device=dev, dtype=torch.float16))
x = torch.randn(1, 1, 4096, device=dev, dtype=torch.float16)
mask = torch.zeros(1, 1, 1, kv + 1, device=dev, dtype=torch.float16)
pos = torch.tensor([[kv]], device=dev)
with torch.no_grad():
    for _ in range(3):
        layer(x, attention_mask=mask, position_ids=pos, past_key_value=past)
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(5):
            layer(x, attention_mask=mask, position_ids=pos, past_key_value=past)
        torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=30, max_name_column_width=60, max_shapes_column_width=60))
