"""End-to-end networks vs eager, forward and backward (reference: ``thunder/tests/test_networks.py``).

Hugging Face ``transformers`` models are built from small random-init configs (no network access)
and acquired by the bytecode interpreter, so these exercise the interpreter on real library code
(decorators, ``**kwargs`` forwarding, ``ModelOutput`` dataclasses, mask helpers, MoE routing).
"""
import pytest
import torch

import lightning_thunder_amd as thunder

tf = pytest.importorskip("transformers")

SMALL = dict(vocab_size=128, hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
             max_position_embeddings=64, use_cache=False)


def _cases():
    c = {
        "llama": ("LlamaConfig", "LlamaForCausalLM", dict(num_key_value_heads=2)),
        "mistral": ("MistralConfig", "MistralForCausalLM", dict(num_key_value_heads=2)),
        "qwen2": ("Qwen2Config", "Qwen2ForCausalLM", dict(num_key_value_heads=2)),
        "phi3": ("Phi3Config", "Phi3ForCausalLM", dict(pad_token_id=0)),
        "gemma": ("GemmaConfig", "GemmaForCausalLM", dict(num_key_value_heads=2, head_dim=16)),
        "gpt2": ("GPT2Config", "GPT2LMHeadModel", dict(n_embd=64, n_layer=2, n_head=4, n_positions=64, resid_pdrop=0.0,
                                                         embd_pdrop=0.0, attn_pdrop=0.0)),
        "bert": ("BertConfig", "BertForMaskedLM", dict(hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)),
        "gpt_neox": ("GPTNeoXConfig", "GPTNeoXForCausalLM", dict()),
        "qwen3_moe": ("Qwen3MoeConfig", "Qwen3MoeForCausalLM", dict(num_experts=4, num_experts_per_tok=2,
                                                                     moe_intermediate_size=32, num_key_value_heads=2)),
    }
    return {k: v for k, v in c.items() if hasattr(tf, v[0]) and hasattr(tf, v[1])}


@pytest.mark.parametrize("name", sorted(_cases()))
def test_hf_causal_lm_training_parity(name):
    cfg_name, model_name, extra = _cases()[name]
    kw = dict(SMALL)
    kw.update(extra)
    torch.manual_seed(0)
    model = getattr(tf, model_name)(getattr(tf, cfg_name)(**kw))
    x = torch.randint(1, 128, (2, 16))
    jm = thunder.jit(model)
    out = jm(x, labels=x)
    ref = model(x, labels=x)
    assert type(out) is type(ref)  # ModelOutput is rebuilt
    torch.testing.assert_close(out.logits, ref.logits)
    torch.testing.assert_close(out.loss, ref.loss)
    out.loss.backward()
    grads = [None if p.grad is None else p.grad.clone() for p in model.parameters()]
    model.zero_grad()
    ref.loss.backward()
    for g, p in zip(grads, model.parameters()):
        if p.grad is None:
            continue
        torch.testing.assert_close(g, p.grad, atol=1e-5, rtol=1e-4)
    # second call hits the cache (prologue guards on config values hold)
    jm(x, labels=x)
    assert thunder.cache_hits(jm) == 1


def test_hf_llama_padding_mask_and_eval_guard():
    cfg = tf.LlamaConfig(**SMALL, num_key_value_heads=2)
    torch.manual_seed(0)
    model = tf.LlamaForCausalLM(cfg)
    x = torch.randint(1, 128, (2, 16))
    mask = torch.ones_like(x)
    mask[1, :5] = 0  # left padding on the second sequence
    jm = thunder.jit(model)
    torch.testing.assert_close(jm(x, attention_mask=mask).logits, model(x, attention_mask=mask).logits)
    model.eval()
    with torch.no_grad():
        torch.testing.assert_close(jm(x, attention_mask=mask).logits, model(x, attention_mask=mask).logits)
    assert thunder.cache_misses(jm) == 2


def test_hf_bart_eval():
    cfg = tf.BartConfig(vocab_size=128, d_model=64, encoder_layers=1, decoder_layers=1, encoder_attention_heads=4,
                        decoder_attention_heads=4, encoder_ffn_dim=64, decoder_ffn_dim=64, max_position_embeddings=64,
                        use_cache=False)
    torch.manual_seed(0)
    model = tf.BartForConditionalGeneration(cfg).eval()
    x = torch.randint(3, 128, (2, 12))
    with torch.no_grad():
        torch.testing.assert_close(thunder.jit(model)(x, labels=x).logits, model(x, labels=x).logits)


@pytest.mark.parametrize("name", ["llama2-like", "codellama2-like", "mistral-like", "falcon-7b-like", "gpt-neox-like",
                                  "gemma-like"])
def test_litgpt_configs_training_parity(name):
    from lightning_thunder_amd.models.litgpt import GPT, Config, init_weights

    try:
        Config.from_name(name)
    except (KeyError, ValueError):
        pytest.skip(f"{name} not a known config")
    torch.manual_seed(0)
    m = GPT.from_name(name)
    init_weights(m)
    m.set_rope_cache(16)
    x = torch.randint(0, 64, (2, 16))
    jm = thunder.jit(m)
    out = jm(x)
    ref = m(x)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-4)
    out.sum().backward()
    grads = [p.grad.clone() for p in m.parameters()]
    m.zero_grad()
    ref.sum().backward()
    for g, p in zip(grads, m.parameters()):
        torch.testing.assert_close(g, p.grad, atol=1e-4, rtol=1e-3)


def test_nanogpt_training_parity():
    from lightning_thunder_amd.models.nanogpt import NanoGPT

    torch.manual_seed(0)
    m = NanoGPT.from_name("gpt2", n_layer=2, n_embd=64, n_head=4, vocab_size=256, block_size=64, dropout=0.0)
    x = torch.randint(0, 256, (2, 32))
    jm = thunder.jit(m)
    logits, loss = jm(x, x)
    rl, rloss = m(x, x)
    torch.testing.assert_close(logits, rl, atol=1e-5, rtol=1e-4)
    loss.backward()
    g = [p.grad.clone() for p in m.parameters()]
    m.zero_grad()
    rloss.backward()
    for a, p in zip(g, m.parameters()):
        torch.testing.assert_close(a, p.grad, atol=1e-5, rtol=1e-4)


def test_nanogpt_dropout_trains():
    from lightning_thunder_amd.models.nanogpt import NanoGPT

    torch.manual_seed(0)
    m = NanoGPT.from_name("test", dropout=0.1, vocab_size=256, block_size=16, n_head=2)
    x = torch.randint(0, 256, (4, 8))
    jm = thunder.jit(m)
    _, loss = jm(x, x)
    loss.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())


def test_hf_generate_static_cache_through_recipe():
    cfg = tf.LlamaConfig(vocab_size=128, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                         num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=128)
    torch.manual_seed(0)
    m = tf.LlamaForCausalLM(cfg).eval()
    m.requires_grad_(False)
    x = torch.randint(1, 128, (1, 8))
    kw = dict(do_sample=False, max_new_tokens=10, min_new_tokens=10, cache_implementation="static", pad_token_id=0)
    ref = m.generate(x, **kw)
    tm = thunder.compile(m, recipe="hf-transformers")
    for _ in range(3):  # every generate() builds a fresh StaticCache: the cached programs must serve it
        out = tm.generate(x, **kw)
        assert torch.equal(out, ref), (out, ref)
    assert thunder.cache_misses(tm) == 2  # one prefill and one decode program
    assert thunder.cache_hits(tm) >= 25
    # repeat_kv is not materialised: SDPA reads the grouped KV cache directly
    comp = [t for t in thunder.last_traces(tm) if "SDPAGQATransform" in str(t.get_provenance())]
    assert comp and "enable_gqa=True" in str(comp[-1]) and "expand(" not in str(comp[-1])


@pytest.mark.parametrize("name", ["llama2-like", "mixtral-like"])
def test_litgpt_init_weights_after_to_empty(name):
    """A model materialised from meta with ``to_empty`` is fully initialised by ``init_weights``:
    norm weights one, expert weights finite and random (benchmarks build models this way)."""
    from lightning_thunder_amd.models.litgpt import GPT, Config, RMSNorm, init_weights

    with torch.device("meta"):
        m = GPT(Config.from_name(name))
    m = m.to_empty(device="cpu")
    for p in m.parameters():
        p.data.fill_(float("nan"))
    init_weights(m)
    for n, p in m.named_parameters():
        assert torch.isfinite(p).all(), n
    norms = [mod for mod in m.modules() if isinstance(mod, (RMSNorm, torch.nn.LayerNorm))]
    assert norms and all(torch.equal(mod.weight, torch.ones_like(mod.weight)) for mod in norms)
    m.set_rope_cache(16, device="cpu")
    idx = torch.randint(0, m.config.vocab_size, (1, 16))
    logits = m(idx)
    assert torch.isfinite(logits).all() and logits.std() > 0


def test_hf_rope_transform_rewrites_attention_prologue():
    """HF rotate-half RoPE on q / k (three projections of one input) -> one concatenated projection
    + the fused split-RoPE op (trace structure; the GPU test runs it)."""
    from lightning_thunder_amd.transforms.hf_rope import HFRoPETransform

    cfg = tf.LlamaConfig(vocab_size=128, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                         num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=128)
    m = tf.LlamaForCausalLM(cfg).eval()
    m.requires_grad_(False)
    comp = thunder.trace(m, torch.randint(1, 128, (1, 8)))
    _, new, _ = HFRoPETransform(require_gpu=False).transform_traces_pre_prologue(None, comp, None)
    s = str(new)
    assert s.count("hip_qkv_rope(") == 2  # one per layer
    assert "ltorch.neg(" not in s  # the rotate_half chains are gone
    # on CPU tensors the transform stays off by default
    _, same, _ = HFRoPETransform().transform_traces_pre_prologue(None, comp, None)
    assert same is comp


def _hf_arch(name):
    import transformers as tf

    ids = torch.randint(0, 100, (2, 12), generator=torch.Generator().manual_seed(0))
    small = dict(vocab_size=100, hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=4,
                 max_position_embeddings=64)
    if name == "gpt2":
        return tf.GPT2LMHeadModel(tf.GPT2Config(vocab_size=100, n_embd=32, n_layer=2, n_head=2, n_positions=64)), {"input_ids": ids}
    if name == "mistral":
        return tf.MistralForCausalLM(tf.MistralConfig(**small, num_key_value_heads=2)), {"input_ids": ids}
    if name == "qwen2":
        return tf.Qwen2ForCausalLM(tf.Qwen2Config(**small, num_key_value_heads=2)), {"input_ids": ids}
    if name == "phi":
        return tf.PhiForCausalLM(tf.PhiConfig(**small)), {"input_ids": ids}
    if name == "gemma":
        return tf.GemmaForCausalLM(tf.GemmaConfig(**small, num_key_value_heads=1, head_dim=8)), {"input_ids": ids}
    if name == "t5":
        cfg = tf.T5Config(vocab_size=100, d_model=32, d_kv=8, d_ff=64, num_layers=2, num_heads=4)
        return tf.T5ForConditionalGeneration(cfg), {"input_ids": ids, "decoder_input_ids": ids[:, :5]}
    if name == "vit":
        cfg = tf.ViTConfig(hidden_size=32, num_hidden_layers=2, num_attention_heads=2, intermediate_size=64, image_size=16,
                           patch_size=4)
        return tf.ViTModel(cfg), {"pixel_values": torch.randn(2, 3, 16, 16, generator=torch.Generator().manual_seed(1))}
    if name == "roberta":
        cfg = tf.RobertaConfig(vocab_size=100, hidden_size=32, num_hidden_layers=2, num_attention_heads=2, intermediate_size=64)
        return tf.RobertaModel(cfg), {"input_ids": ids}
    if name == "mixtral":
        return tf.MixtralForCausalLM(tf.MixtralConfig(**small, num_key_value_heads=2, num_local_experts=4,
                                                      num_experts_per_tok=2)), {"input_ids": ids}
    if name == "falcon":
        return tf.FalconForCausalLM(tf.FalconConfig(vocab_size=100, hidden_size=32, num_hidden_layers=2,
                                                    num_attention_heads=4)), {"input_ids": ids}
    raise ValueError(name)


@pytest.mark.parametrize("name", ["gpt2", "mistral", "qwen2", "phi", "gemma", "t5", "vit", "roberta", "mixtral", "falcon"])
def test_hf_architectures_fwd_bwd(name):
    """HF transformers architectures through the interpreter: outputs and parameter gradients
    match eager (reference analogue: thunder/tests/test_networks.py HF model tests).  hipfuse
    partitions the CPU program too (its regions run the reference path) and every generated
    kernel is compiled for gfx950 with hiprtc."""
    import os

    from lightning_thunder_amd.executors import hipfuse

    torch.manual_seed(0)
    model, inputs = _hf_arch(name)
    model.eval()
    key = "logits" if hasattr(model, "lm_head") or name == "t5" else "last_hidden_state"
    ref = getattr(model(**inputs), key)
    ref.float().pow(2).mean().backward()
    ref_grads = {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
    model.zero_grad()
    old = hipfuse.ex.allow_cpu
    hipfuse.ex.allow_cpu = True
    try:
        jm = thunder.jit(model)
        out = getattr(jm(**inputs), key)
        torch.testing.assert_close(out, ref, atol=1e-4, rtol=1e-4)
        out.float().pow(2).mean().backward()
    finally:
        hipfuse.ex.allow_cpu = old
    for n, g in ref_grads.items():
        p = dict(model.named_parameters())[n]
        torch.testing.assert_close(p.grad, g, atol=1e-4, rtol=1e-3, msg=n)
    if os.path.exists("/opt/rocm/lib/libhiprtc.so"):
        for tr in (thunder.last_traces(jm)[-1], thunder.last_backward_traces(jm)[-1]):
            hipfuse.precompile(tr)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["gpt2", "mistral", "qwen2", "phi", "gemma", "t5", "vit", "roberta", "mixtral", "falcon"])
def test_hf_architectures_gpu_bf16(name):
    """The same architectures in bf16 on the MI355X with the HIP executors claiming what they can
    (flash attention, RMSNorm / LayerNorm, GEMMs, fused elementwise): close to eager bf16."""
    torch.manual_seed(0)
    model, inputs = _hf_arch(name)
    model = model.to("cuda", torch.bfloat16).eval()
    inputs = {k: (v.to("cuda", torch.bfloat16) if v.is_floating_point() else v.cuda()) for k, v in inputs.items()}
    key = "logits" if hasattr(model, "lm_head") or name == "t5" else "last_hidden_state"
    ref = getattr(model(**inputs), key).float()
    ref.pow(2).mean().backward()
    ref_grads = {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}
    model.zero_grad()
    out = getattr(thunder.jit(model)(**inputs), key).float()
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 3e-2, rel
    out.pow(2).mean().backward()
    scale = max(g.norm().item() for g in ref_grads.values())
    for n, g in ref_grads.items():
        p = dict(model.named_parameters())[n]
        if g.norm() < 1e-3 * scale:
            continue  # e.g. attention key biases: exactly zero in exact arithmetic (softmax shift invariance)
        cos = torch.nn.functional.cosine_similarity(p.grad.float().flatten(), g.flatten(), dim=0).item()
        assert cos > 0.98, (n, cos)
