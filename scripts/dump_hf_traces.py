"""Dump the HF Llama decode program (compile(recipe='hf-transformers', plugins='reduce-overhead'))."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.benchmarks.generate import _build_hf

out_dir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/hf_traces"
os.makedirs(out_dir, exist_ok=True)
model, cfg = _build_hf(torch.device("cuda", 0), n_layer=2)
gm = thunder.compile(model, recipe="hf-transformers", plugins="reduce-overhead")
prompt = torch.randint(1, cfg.vocab_size, (1, 16), device="cuda")
kw = dict(max_new_tokens=4, min_new_tokens=4, do_sample=False, cache_implementation="static", pad_token_id=0,
          disable_compile=True)
gm.generate(prompt, **kw)
traces = thunder.last_traces(gm)
with open(os.path.join(out_dir, "decode_final.py"), "w") as f:
    f.write(str(traces[-1]))
with open(os.path.join(out_dir, "decode_first.py"), "w") as f:
    f.write(str(traces[0]))
with open(os.path.join(out_dir, "decode_pregraph.py"), "w") as f:
    f.write(str(traces[-2]))
print("ok", len(traces))
