"""LoRA / QLoRA / QA-LoRA / ReLoRA / LISA fine-tuning on CPU, FusedAdamW vs
torch.optim.AdamW, adapter save/load, merge, DDP (gloo) consistency.
Reference: example/GPU/LLM-Finetuning (QLoRA, QA-LoRA, ReLoRA, LISA)."""
import os

import pytest
import torch


def _model(tmp_path, qtype="sym_int4"):
    from transformers import LlamaConfig, LlamaForCausalLM
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=128, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256)
    p = str(tmp_path / "base")
    if not os.path.exists(p):
        LlamaForCausalLM(cfg).save_pretrained(p)
    return AutoModelForCausalLM.from_pretrained(p, load_in_low_bit=qtype, optimize_model=False,
                                                torch_dtype=torch.float32, modules_to_not_convert=["lm_head"])


def _train(model, steps=12, lr=5e-3):
    from ipex_llm_amd.training import FusedAdamW
    opt = FusedAdamW([p for p in model.parameters() if p.requires_grad], lr=lr, weight_decay=0.0)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, 128, (4, 16), generator=g)
    losses = []
    for _ in range(steps):
        out = model(input_ids=ids, labels=ids)
        out.loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(out.loss.item())
    return losses, ids


@pytest.mark.parametrize("mode", ["qlora", "qalora", "lora"])
def test_lora_training_reduces_loss(tmp_path, mode):
    from ipex_llm_amd.training import LoraConfig, get_peft_model, prepare_model_for_kbit_training
    model = _model(tmp_path, "bf16" if mode == "lora" else "sym_int4")
    model = prepare_model_for_kbit_training(model, use_gradient_checkpointing=False)
    pm = get_peft_model(model, LoraConfig(r=8, lora_alpha=16, target_modules=["q_proj", "v_proj", "down_proj"],
                                          training_mode=mode))
    tr, tot = pm.get_nb_trainable_parameters()
    assert 0 < tr < tot
    losses, ids = _train(pm)
    assert losses[-1] < losses[0] - 0.05, losses
    # adapter round trip
    pm.save_pretrained(str(tmp_path / "adapter"))
    from ipex_llm_amd.training import PeftModel
    fresh = _model(tmp_path, "bf16" if mode == "lora" else "sym_int4")
    pm2 = PeftModel.from_pretrained(fresh, str(tmp_path / "adapter"))
    with torch.no_grad():
        a = pm(input_ids=ids).logits
        b = pm2(input_ids=ids).logits
    assert torch.allclose(a, b, atol=1e-4)
    with pm2.disable_adapter(), torch.no_grad():
        c = pm2(input_ids=ids).logits
    assert not torch.allclose(a, c, atol=1e-3)
    merged = pm2.merge_and_unload()
    with torch.no_grad():
        d = merged(input_ids=ids).logits
    tol = 1e-2 if mode == "lora" else 0.15     # bf16 rounding / low-bit re-quantization
    assert ((d - a).norm() / a.norm()).item() < tol


def test_fused_adamw_matches_torch_cpu():
    from ipex_llm_amd.training import FusedAdamW
    torch.manual_seed(0)
    p1 = [torch.nn.Parameter(torch.randn(37, 5)), torch.nn.Parameter(torch.randn(100))]
    p2 = [torch.nn.Parameter(p.detach().clone()) for p in p1]
    o1 = FusedAdamW(p1, lr=1e-2, weight_decay=0.1)
    o2 = torch.optim.AdamW(p2, lr=1e-2, weight_decay=0.1)
    for _ in range(5):
        for a, b in zip(p1, p2):
            g = torch.randn_like(a)
            a.grad, b.grad = g.clone(), g.clone()
        o1.step()
        o2.step()
    for a, b in zip(p1, p2):
        assert torch.allclose(a, b, atol=1e-6)


def test_relora_restart_and_scheduler(tmp_path):
    from ipex_llm_amd.training import FusedAdamW, LoraConfig, get_peft_model, relora_restart, ReLoRAScheduler
    pm = get_peft_model(_model(tmp_path), LoraConfig(r=4, target_modules=["q_proj"], training_mode="relora"))
    losses, ids = _train(pm, steps=6)
    with torch.no_grad():
        before = pm(input_ids=ids).logits
    opt = FusedAdamW([p for p in pm.parameters() if p.requires_grad])
    n = relora_restart(pm, opt)
    assert n == 2
    with torch.no_grad():
        after = pm(input_ids=ids).logits            # merged into the base; adapters restarted (B = 0)
    assert ((after - before).norm() / before.norm()).item() < 0.1
    for m in pm.lora_modules().values():
        assert torch.count_nonzero(m.lora_B.weight) == 0
    sch = ReLoRAScheduler(torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=1.0), 100, 20, 5, 5)
    lrs = []
    for _ in range(30):
        lrs.append(sch.get_last_lr()[0])
        sch.optimizer.step()
        sch.step()
    assert lrs[0] == 0 and lrs[20] < lrs[19]          # re-warmup after the restart


def test_lisa_switches_layers(tmp_path):
    from ipex_llm_amd.training import LayerActivation
    m = _model(tmp_path, "bf16")
    act = LayerActivation(m, n_layers=1, interval_steps=2)
    a = act.maybe_switch(0)
    assert len(a) == 1
    on = [any(p.requires_grad for p in L.parameters()) for L in m.model.layers]
    assert sum(on) == 1
    assert act.maybe_switch(1) is None


def _ddp_worker(rank, world, port, path):
    import os as _os
    _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.training import FusedAdamW, LoraConfig, get_peft_model, wrap_ddp
    m = AutoModelForCausalLM.from_pretrained(path, load_in_low_bit="sym_int4", optimize_model=False,
                                             torch_dtype=torch.float32)
    pm = get_peft_model(m, LoraConfig(r=4, target_modules=["q_proj", "v_proj"]))
    torch.manual_seed(0)
    for mod in pm.lora_modules().values():
        mod.reset_lora_parameters()
    ddp = wrap_ddp(pm)
    opt = FusedAdamW([p for p in ddp.parameters() if p.requires_grad], lr=1e-2)
    ids = torch.randint(0, 128, (2, 12), generator=torch.Generator().manual_seed(rank))
    for _ in range(3):
        loss = ddp(input_ids=ids, labels=ids).loss
        loss.backward()
        opt.step()
        opt.zero_grad()
    v = torch.cat([p.detach().flatten() for p in pm.parameters() if p.requires_grad])
    vs = [torch.empty_like(v) for _ in range(world)]
    dist.all_gather(vs, v)
    assert torch.allclose(vs[0], vs[1]), "replicas diverged"
    dist.destroy_process_group()


def test_ddp_lora_replicas_stay_identical(tmp_path):
    from tests.test_distributed import _free_port
    import torch.multiprocessing as mp
    _model(tmp_path)
    port = _free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_ddp_worker, args=(r, 2, port, str(tmp_path / "base"))) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    assert [p.exitcode for p in ps] == [0, 0]


def _bucket_worker(rank, world, port):
    import os as _os
    _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import copy
    import torch.distributed as dist
    import torch.nn as nn
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ipex_llm_amd.training import FusedAdamW
    from ipex_llm_amd.training.ddp import GradBucketSync
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(16, 32), nn.Tanh(), nn.Linear(32, 32), nn.Tanh(), nn.Linear(32, 4))
    model[2].weight.requires_grad_(False)               # a frozen base weight, like QLoRA
    ref = copy.deepcopy(model)
    if rank == 1:                                       # different init: broadcast must fix it
        with torch.no_grad():
            for p in model.parameters():
                if p.requires_grad:
                    p.add_(1.0)
    sync = GradBucketSync(model, bucket_cap_mb=0.0002)  # ~200 B buckets: several per step
    assert len(sync.buckets) > 2
    sync.broadcast_parameters()
    opt = FusedAdamW([p for p in model.parameters() if p.requires_grad], lr=1e-2)
    ropt = torch.optim.AdamW([p for p in ref.parameters() if p.requires_grad], lr=1e-2, weight_decay=1e-2)
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(world, 5, 16, generator=g) for _ in range(3)]
    for it in range(3):
        x = xs[it]
        model(x[rank]).pow(2).mean().backward()
        sync.finish()
        # reference: the full batch on one replica (mean over ranks of the per-rank means)
        sum(ref(x[r]).pow(2).mean() for r in range(world)).div(world).backward()
        for p, q in zip(model.parameters(), ref.parameters()):
            if p.requires_grad:
                assert torch.allclose(p.grad, q.grad, atol=1e-6), it
        opt.step()
        ropt.step()
        sync.zero_grad()
        ropt.zero_grad()
    # gradient accumulation: 2 micro-batches per step, the first under no_sync()
    for it in range(2):
        x = xs[it]
        with sync.no_sync():
            model(x[rank, :2]).pow(2).mean().div(2).backward()
        model(x[rank, 2:]).pow(2).mean().div(2).backward()
        sync.finish()
        sum(ref(x[r, :2]).pow(2).mean().div(2) + ref(x[r, 2:]).pow(2).mean().div(2)
            for r in range(world)).div(world).backward()
        for p, q in zip(model.parameters(), ref.parameters()):
            if p.requires_grad:
                assert torch.allclose(p.grad, q.grad, atol=1e-6), ("accum", it)
        opt.step()
        ropt.step()
        sync.zero_grad()
        ropt.zero_grad()
    # a second synced backward before finish() must raise, not race
    model(xs[0][rank]).pow(2).mean().backward()
    try:
        model(xs[0][rank]).pow(2).mean().backward()
        raised = False
    except RuntimeError:
        raised = True
    assert raised
    sync.finish()
    sync.zero_grad()
    v = torch.cat([p.detach().flatten() for p in model.parameters() if p.requires_grad])
    vs = [torch.empty_like(v) for _ in range(world)]
    dist.all_gather(vs, v)
    assert torch.allclose(vs[0], vs[1]), "replicas diverged"
    dist.destroy_process_group()


def test_grad_bucket_sync_matches_full_batch():
    """GradBucketSync (flat gradient buffer, per-bucket async all-reduce fired
    from post-accumulate hooks) == full-batch gradients; replicas identical"""
    from tests.test_distributed import _free_port
    import torch.multiprocessing as mp
    port = _free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_bucket_worker, args=(r, 2, port)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    assert [p.exitcode for p in ps] == [0, 0]


@pytest.mark.parametrize("bias", [False, True])
def test_fused_lora_node_matches_module_graph(monkeypatch, bias):
    """the one-node QLoRA linear (LoRA term accumulated into the base GEMM
    output and into grad_x) == base + B(A(x)) * s built module by module"""
    import ipex_llm_amd.training.lora as L
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    torch.manual_seed(1)
    lin = torch.nn.Linear(256, 192, bias=bias)
    base = LowBitLinear.from_linear(lin, "sym_int4")
    if bias:
        base.bias.data = base.bias.data.to(torch.bfloat16)
    lay = L.LoraLinear(base, r=8, alpha=16)
    torch.nn.init.normal_(lay.lora_B.weight, std=0.05)
    x0 = torch.randn(2, 5, 256).to(torch.bfloat16)
    gy = torch.randn(2, 5, 192).to(torch.bfloat16)
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(L, "_FUSED", fused)
        assert lay._fused_ok(x0.clone().requires_grad_()) == fused
        x = x0.clone().requires_grad_()
        lay.zero_grad()
        y = lay(x)
        y.backward(gy)
        res[fused] = (y.float(), x.grad.float(), lay.lora_A.weight.grad.float(), lay.lora_B.weight.grad.float())
    for a, b in zip(res[True], res[False]):
        assert a.shape == b.shape
        assert ((a - b).norm() / b.norm()).item() < 2e-2


def test_reference_qlora_class_names():
    """ipex_llm.transformers.qlora names: LoraLowBitLinear over a low-bit
    base, LoraBF16Linear over a dense bf16 base, each refusing the other"""
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    from ipex_llm_amd.transformers.qlora import LoraBF16Linear, LoraLowBitLinear
    lin = torch.nn.Linear(128, 64, bias=False)
    low = LowBitLinear.from_linear(lin, "nf4")
    a = LoraLowBitLinear(low, r=4, lora_alpha=8)
    b = LoraBF16Linear(torch.nn.Linear(128, 64, bias=False), r=4, lora_alpha=8)
    x = torch.randn(3, 128).to(torch.bfloat16)
    assert a(x).shape == (3, 64) and b(x).shape == (3, 64)
    assert b.base_layer.weight.dtype == torch.bfloat16
    with pytest.raises(TypeError):
        LoraLowBitLinear(lin)
    with pytest.raises(TypeError):
        LoraBF16Linear(low)


def test_fused_adamw_state_dict_round_trip_keeps_step():
    """state_dict() carries the step count (bias correction) and a resumed
    optimizer continues exactly where the original one was"""
    from ipex_llm_amd.training import FusedAdamW
    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(64))
    opt = FusedAdamW([p], lr=1e-2)
    for _ in range(3):
        p.grad = torch.randn(64)
        opt.step()
    sd = opt.state_dict()
    assert sd["state"][0]["step"] == 3
    q = torch.nn.Parameter(p.detach().clone())
    opt2 = FusedAdamW([q], lr=1e-2)
    import copy
    opt2.load_state_dict(copy.deepcopy(sd))     # as from disk (torch keeps the moment tensors otherwise)
    g = torch.randn(64)
    p.grad, q.grad = g.clone(), g.clone()
    opt.step()
    opt2.step()
    assert torch.allclose(p, q) and opt2.state[q]["step"] == 4


def test_grouped_lora_siblings_match_per_module(monkeypatch):
    """q/k/v and gate/up adapters over one input as one _LoraGroupFn node ==
    the per-module fused nodes: outputs, grad_x and every adapter gradient"""
    import torch.nn as nn
    from ipex_llm_amd.training import lora as L
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear

    class Blk(nn.Module):
        def __init__(self):
            super().__init__()
            for n, o in (("q_proj", 256), ("k_proj", 128), ("v_proj", 128), ("gate_proj", 384), ("up_proj", 384)):
                m = LowBitLinear(256, o, "sym_int8", bias=False, device="meta")
                m.load_dense(torch.randn(o, 256) * 0.05, device="cpu")
                setattr(self, n, m)

        def forward(self, x):
            return (self.q_proj(x).sum() + 2 * self.k_proj(x).sum() + (self.v_proj(x) ** 2).sum()
                    + (self.gate_proj(x) * self.up_proj(x)).sum())

    torch.manual_seed(0)
    blk = Blk()
    model = L.get_peft_model(blk, L.LoraConfig(r=4, lora_alpha=8, target_modules=["q_proj", "k_proj", "v_proj",
                                                                                     "gate_proj", "up_proj"]))
    assert L.link_lora_groups(blk) == 2
    for m in model.lora_modules().values():
        m.to(torch.bfloat16)
        with torch.no_grad():
            m.lora_B.weight.normal_(0, 0.05)
    x0 = torch.randn(2, 7, 256, dtype=torch.bfloat16)

    def run(group):
        monkeypatch.setattr(L, "_GROUP", group)
        calls = []
        orig = L._LoraGroupFn.forward
        monkeypatch.setattr(L._LoraGroupFn, "forward", staticmethod(lambda *a: calls.append(1) or orig(*a)))
        for p in model.parameters():
            p.grad = None
        x = x0.clone().requires_grad_(True)
        out = blk(x)
        out.backward()
        grads = {n: p.grad.float().clone() for n, p in model.named_parameters() if p.requires_grad}
        return out.float(), x.grad.float(), grads, len(calls)
    o1, gx1, g1, n1 = run(True)
    o0, gx0, g0, n0 = run(False)
    assert n1 == 2 and n0 == 0
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()      # noqa: E731  (bf16 summation order differs)
    assert rel(o1, o0) < 1e-2
    assert rel(gx1, gx0) < 2e-2
    for k in g0:
        assert rel(g1[k], g0[k]) < 2e-2, k


def test_fused_ce_refuses_softcap_and_scaled_heads():
    """heads whose HF loss soft-caps or scales the logits keep the HF forward
    (the fused lm_head + CE applies neither)"""
    from types import SimpleNamespace
    from ipex_llm_amd.training.fused_ce import plain_ce_head
    assert plain_ce_head(None)
    assert plain_ce_head(SimpleNamespace(final_logit_softcapping=None, logit_scale=None))
    assert not plain_ce_head(SimpleNamespace(final_logit_softcapping=30.0))
    assert not plain_ce_head(SimpleNamespace(logit_scale=0.0625))
    assert not plain_ce_head(SimpleNamespace(logits_scaling=8.0))
    assert plain_ce_head(SimpleNamespace(logits_scaling=1.0))


def test_link_lora_groups_skips_cross_attention():
    """q / k / v of a cross-attention block read different inputs: never grouped"""
    import torch.nn as nn
    from ipex_llm_amd.training.lora import LoraConfig, get_peft_model, link_lora_groups

    class Attn(nn.Module):
        def __init__(self):
            super().__init__()
            self.q_proj, self.k_proj, self.v_proj = nn.Linear(64, 64), nn.Linear(64, 64), nn.Linear(64, 64)

    class Layer(nn.Module):
        def __init__(self):
            super().__init__()
            self.self_attn, self.encoder_attn = Attn(), Attn()

    m = nn.Sequential(Layer())
    peft = get_peft_model(m, LoraConfig(r=4, target_modules=["q_proj", "k_proj", "v_proj"]))
    assert link_lora_groups(peft) == 1
    assert "_lora_group" in m[0].self_attn.q_proj.__dict__
    assert "_lora_group" not in m[0].encoder_attn.q_proj.__dict__


def test_rotary_patch_matches_hf():
    """the training rotary-embedding patch (broadcast multiply instead of the
    K = 1 f32 matmul) returns HF's cos / sin bit for bit"""
    from transformers import LlamaConfig
    from transformers.models.llama.modeling_llama import LlamaRotaryEmbedding
    from ipex_llm_amd.training.lora import _patch_rotary
    cfg = LlamaConfig(hidden_size=256, num_attention_heads=4, max_position_embeddings=512, rope_theta=500000.0)
    holder = torch.nn.Module()
    holder.rotary_emb = LlamaRotaryEmbedding(cfg)
    x = torch.randn(2, 7, 256, dtype=torch.bfloat16)
    pos = torch.tensor([[0, 1, 2, 3, 4, 5, 6], [10, 11, 12, 300, 301, 302, 511]])
    c0, s0 = holder.rotary_emb(x, pos)
    assert _patch_rotary(holder) == 1
    c1, s1 = holder.rotary_emb(x, pos)
    assert torch.equal(c0, c1) and torch.equal(s0, s1)


def test_rotary_patch_skips_mrope():
    """Qwen2-VL's text rotary reports rope_type 'default' but takes 3-D M-RoPE
    positions [3, bs, seq]: the patch leaves it alone, and a
    patched rotary handed non-2-D positions falls back to its own forward"""
    from transformers import Qwen2VLConfig
    from transformers.models.qwen2_vl.modeling_qwen2_vl import Qwen2VLRotaryEmbedding
    from ipex_llm_amd.training.lora import _patch_rotary
    cfg = Qwen2VLConfig(hidden_size=256, num_attention_heads=4, num_key_value_heads=4,
                        rope_scaling={"type": "mrope", "mrope_section": [8, 12, 12]})
    tc = getattr(cfg, "text_config", cfg)
    holder = torch.nn.Module()
    holder.rotary_emb = Qwen2VLRotaryEmbedding(tc)
    x = torch.randn(2, 5, 256, dtype=torch.bfloat16)
    pos = torch.arange(5).view(1, 1, 5).expand(3, 2, 5).contiguous()
    c0, s0 = holder.rotary_emb(x, pos)
    _patch_rotary(holder)
    c1, s1 = holder.rotary_emb(x, pos)
    assert c1.shape == c0.shape and torch.equal(c0, c1) and torch.equal(s0, s1)


def test_relora_merge_and_save_resume_reproduces_uninterrupted(tmp_path):
    """ReLoRA merged full-weight checkpoints (reference relora.py:383-471):
    train -> restart through merge_and_save -> train; a fresh model that
    resumes from the save (load_weight_checkpoint) + the adapter checkpoint
    holds exactly the uninterrupted run's low-bit base and adapters, and the
    saved shards are the fp16 full weights + the merged deltas"""
    from safetensors.torch import load_file
    from ipex_llm_amd.training import (LoraConfig, get_peft_model, load_weight_checkpoint, merge_and_save,
                                       find_lora_modules)
    from ipex_llm_amd.training.lora import PeftModel
    cfg = LoraConfig(r=4, lora_alpha=8, target_modules=["q_proj", "v_proj"], training_mode="relora")
    pm = get_peft_model(_model(tmp_path), cfg)
    _train(pm, steps=3)
    src = str(tmp_path / "base")
    base_sd = load_file(os.path.join(src, "model.safetensors"))
    deltas = {n + ".weight": m.delta_weight().clone() for n, m in find_lora_modules(pm).items()}
    dst = str(tmp_path / "ckpt-3" / "relora")
    merge_and_save(pm, src, dst, reinit=True)
    saved = load_file(os.path.join(dst, "model.safetensors"))
    assert set(saved) == set(base_sd)
    for k, d in deltas.items():
        assert torch.equal(saved[k], (base_sd[k].float() + d).half())
    for m in find_lora_modules(pm).values():                      # restarted adapters
        assert torch.count_nonzero(m.lora_B.weight) == 0
    # the checkpoint a resumed job would have: adapters right after the restart
    pm.save_pretrained(str(tmp_path / "adapter"))
    _train(pm, steps=2)                                           # the uninterrupted run continues
    # resume: fresh model from the ORIGINAL checkpoint + the merged save + adapters
    fresh = PeftModel.from_pretrained(_model(tmp_path), str(tmp_path / "adapter"), is_trainable=True)
    assert load_weight_checkpoint(fresh, dst) == len(deltas)
    _train(fresh, steps=2)
    a, b = find_lora_modules(pm), find_lora_modules(fresh)
    for n in a:
        assert torch.equal(a[n].base_layer.weight, b[n].base_layer.weight), n
        assert torch.allclose(a[n].lora_A.weight, b[n].lora_A.weight, atol=1e-6), n
        assert torch.allclose(a[n].lora_B.weight, b[n].lora_B.weight, atol=1e-6), n


def test_relora_callback_writes_and_resumes(tmp_path):
    """the HF callback: merge_and_save into checkpoint-<step>/relora at each
    restart, on_train_begin resumes from it"""
    from types import SimpleNamespace
    from ipex_llm_amd.training import LoraConfig, get_peft_model
    from ipex_llm_amd.training.relora import ReLoRACallback, find_lora_modules
    pm = get_peft_model(_model(tmp_path), LoraConfig(r=4, target_modules=["q_proj"], training_mode="relora"))
    _train(pm, steps=2)
    cb = ReLoRACallback(relora_steps=2, base_model=str(tmp_path / "base"))
    args = SimpleNamespace(output_dir=str(tmp_path / "out"), process_index=0)
    cb.on_step_begin(args, SimpleNamespace(global_step=2), None, model=pm, optimizer=None)
    path = tmp_path / "out" / "checkpoint-2" / "relora" / "model.safetensors"
    assert path.exists() and cb.restarts == 1
    fresh = get_peft_model(_model(tmp_path), LoraConfig(r=4, target_modules=["q_proj"], training_mode="relora"))
    ReLoRACallback(relora_steps=2, base_model=str(tmp_path / "base"),
                   resume_from_checkpoint=str(tmp_path / "out" / "checkpoint-2")).on_train_begin(args, None, None,
                                                                                                 model=fresh)
    for n, m in find_lora_modules(pm).items():
        assert torch.equal(m.base_layer.weight, find_lora_modules(fresh)[n].base_layer.weight)
