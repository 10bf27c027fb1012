"""GGUF import/export (reference gguf/gguf.py dequantizers, gguf/api.py
builders).  No GGUF fixtures ship with the reference, so files are written
by our own writer; k-quant dequantizers are checked against a direct scalar
transcription of the ggml block loops (parity unpinned vs llama.cpp itself)."""
import numpy as np
import pytest
import torch

from ipex_llm_amd.gguf import reader as G


def _tiny(tmp_path):
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512)
    m = LlamaForCausalLM(cfg).eval()
    p = str(tmp_path / "hf")
    m.save_pretrained(p)
    return m, p


@pytest.mark.parametrize("qt,tol", [("f32", 1e-5), ("q8_0", 2e-2), ("q4_0", 0.2)])
def test_gguf_export_import_roundtrip(tmp_path, qt, tol):
    from ipex_llm_amd.convert_model import llm_convert
    from ipex_llm_amd.gguf.api import load_gguf_model
    ref, p = _tiny(tmp_path)
    f = llm_convert(p, str(tmp_path / f"m-{qt}.gguf"), f"gguf_{qt}")
    r = G.GGUFReader(f)
    assert r.architecture == "llama" and r.kv["llama.block_count"] == 2
    m, tok = load_gguf_model(f, dtype=torch.float32)
    ids = torch.randint(0, 256, (2, 9))
    with torch.no_grad():
        a, b = ref(ids).logits, m(ids).logits
    assert ((a - b).norm() / a.norm()).item() < tol


def test_from_gguf_low_bit(tmp_path):
    from ipex_llm_amd.convert_model import export_gguf
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    ref, p = _tiny(tmp_path)
    f = export_gguf(ref, str(tmp_path / "m.gguf"), "f16")
    m, _ = AutoModelForCausalLM.from_gguf(f, low_bit="sym_int8")
    ids = torch.randint(0, 256, (1, 7))
    with torch.no_grad():
        a, b = ref(ids).logits, m(ids).logits.float()
    assert ((a - b).norm() / a.norm()).item() < 5e-2
    assert m.generate(ids, max_new_tokens=3).shape == (1, 10)


def _scale_min_k4(j, q):
    if j < 4:
        return q[j] & 63, q[j + 4] & 63
    return (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4), (q[j + 4] >> 4) | ((q[j] >> 6) << 4)


def _ref_q4k(b):
    d = np.frombuffer(bytes(b[0:2]), np.float16)[0].astype(np.float32)
    dmin = np.frombuffer(bytes(b[2:4]), np.float16)[0].astype(np.float32)
    sc, qs = b[4:16], b[16:144]
    y, is_, q = [], 0, 0
    for j in range(0, 256, 64):
        s1, m1 = _scale_min_k4(is_, sc)
        s2, m2 = _scale_min_k4(is_ + 1, sc)
        y += [d * s1 * (qs[q + l] & 0xF) - dmin * m1 for l in range(32)]
        y += [d * s2 * (qs[q + l] >> 4) - dmin * m2 for l in range(32)]
        q += 32
        is_ += 2
    return np.array(y, np.float32)


def _ref_q5k(b):
    d = np.frombuffer(bytes(b[0:2]), np.float16)[0].astype(np.float32)
    dmin = np.frombuffer(bytes(b[2:4]), np.float16)[0].astype(np.float32)
    sc, qh, ql = b[4:16], b[16:48], b[48:176]
    y, is_, q, u1, u2 = [], 0, 0, 1, 2
    for j in range(0, 256, 64):
        s1, m1 = _scale_min_k4(is_, sc)
        s2, m2 = _scale_min_k4(is_ + 1, sc)
        y += [d * s1 * ((ql[q + l] & 0xF) + (16 if qh[l] & u1 else 0)) - dmin * m1 for l in range(32)]
        y += [d * s2 * ((ql[q + l] >> 4) + (16 if qh[l] & u2 else 0)) - dmin * m2 for l in range(32)]
        q += 32
        is_ += 2
        u1 <<= 2
        u2 <<= 2
    return np.array(y, np.float32)


def _ref_q6k(b):
    ql, qh = b[0:128], b[128:192]
    sc = np.frombuffer(bytes(b[192:208]), np.int8).astype(np.float32)
    d = np.frombuffer(bytes(b[208:210]), np.float16)[0].astype(np.float32)
    y = np.zeros(256, np.float32)
    for n in range(2):
        for l in range(32):
            is_ = l // 16
            L, H, S = ql[64 * n:], qh[32 * n:], sc[8 * n:]
            q1 = ((L[l] & 0xF) | (((H[l] >> 0) & 3) << 4)) - 32
            q2 = ((L[l + 32] & 0xF) | (((H[l] >> 2) & 3) << 4)) - 32
            q3 = ((L[l] >> 4) | (((H[l] >> 4) & 3) << 4)) - 32
            q4 = ((L[l + 32] >> 4) | (((H[l] >> 6) & 3) << 4)) - 32
            y[128 * n + l] = d * S[is_] * q1
            y[128 * n + l + 32] = d * S[is_ + 2] * q2
            y[128 * n + l + 64] = d * S[is_ + 4] * q3
            y[128 * n + l + 96] = d * S[is_ + 6] * q4
    return y


@pytest.mark.parametrize("t,ref", [(G.Q4_K, _ref_q4k), (G.Q5_K, _ref_q5k), (G.Q6_K, _ref_q6k)])
def test_kquant_dequant_matches_scalar_loops(t, ref):
    rng = np.random.default_rng(0)
    be, bb = G.BLOCK[t]
    raw = rng.integers(0, 256, size=3 * bb, dtype=np.uint8)
    # sane fp16 scales (avoid inf/nan bit patterns)
    for i in range(3):
        blk = raw[i * bb:(i + 1) * bb]
        if t == G.Q6_K:
            blk[208:210] = np.frombuffer(np.float16(0.01).tobytes(), np.uint8)
        else:
            blk[0:2] = np.frombuffer(np.float16(0.02).tobytes(), np.uint8)
            blk[2:4] = np.frombuffer(np.float16(0.005).tobytes(), np.uint8)
    got = G.dequantize(raw, t, 3 * be)
    want = np.concatenate([ref(raw[i * bb:(i + 1) * bb].tolist()) for i in range(3)])
    assert np.allclose(got, want, atol=1e-5)


@pytest.mark.parametrize("t", [G.Q4_0, G.Q8_0])
def test_legacy_quant_roundtrip(t):
    x = np.random.default_rng(1).standard_normal(256).astype(np.float32)
    raw = np.frombuffer(G.quantize_q4_0(x) if t == G.Q4_0 else G.quantize_q8_0(x), np.uint8)
    y = G.dequantize(raw, t, 256)
    assert np.abs(y - x).max() < (0.5 if t == G.Q4_0 else 0.03)


@pytest.mark.parametrize("qt", ["q4_k", "q4_k_m", "q6_k", "q2_k"])
def test_from_gguf_keeps_kquant_blocks(tmp_path, qt):
    """k-quant GGUF tensors load as KQuantLinear over the file's own blocks
    (no dequantize / re-quantize): bits per weight and numerics equal the
    file's -- logits match a dense model built from the dequantized tensors"""
    from ipex_llm_amd.convert_model import export_gguf
    from ipex_llm_amd.gguf.api import load_gguf_model
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.transformers.low_bit_linear import KQuantLinear, RowConcatLinear
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=256, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512)
    ref = LlamaForCausalLM(cfg).eval()
    f = export_gguf(ref, str(tmp_path / f"m-{qt}.gguf"), qt)
    r = G.GGUFReader(f)
    kinds = {r.tensors[n].ggml_type for n in r.tensors if n.endswith("attn_v.weight") or n.endswith("ffn_up.weight")}
    assert kinds & {G.Q2_K, G.Q4_K, G.Q5_K, G.Q6_K}
    dense, _ = load_gguf_model(f, dtype=torch.float32)                 # dequantized reference
    m, _ = AutoModelForCausalLM.from_gguf(f, low_bit="sym_int8", keep_kquant=True, torch_dtype=torch.float32)
    kq = [x for x in m.modules() if isinstance(x, (KQuantLinear, RowConcatLinear))]
    assert kq, "no k-quant module kept"
    if qt == "q4_k_m":       # v rows in q6_k, q/k in q4_k: the merged qkv keeps both types
        assert any(isinstance(x, RowConcatLinear) for x in kq)
    ids = torch.randint(0, 256, (1, 9))
    with torch.no_grad():
        a = dense(ids).logits
        b = m(ids).logits.float()
        # the CPU k-quant GEMM multiplies int8 activations (per-64 scales) against
        # the super-block codes, as ggml's q8 x k-quant dot does
        assert ((a - b).norm() / a.norm()).item() < 3e-2


def _family(kind):
    import transformers as T
    if kind == "bloom":
        return T.BloomConfig(vocab_size=256, hidden_size=256, n_layer=2, n_head=4)
    if kind == "falcon":
        return T.FalconConfig(vocab_size=256, hidden_size=256, num_hidden_layers=2, num_attention_heads=4)
    if kind == "falcon_new":
        return T.FalconConfig(vocab_size=256, hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
                              num_kv_heads=2, new_decoder_architecture=True)
    return T.MptConfig(vocab_size=256, d_model=256, n_layers=2, n_heads=4, max_seq_len=256)


@pytest.mark.parametrize("kind", ["bloom", "falcon", "falcon_new", "mpt"])
@pytest.mark.parametrize("qt", ["f16", "q4_k"])
def test_gguf_family_round_trip(tmp_path, kind, qt):
    """bloom / falcon / mpt through llama.cpp's tensor names and [q; k; v]
    fused-QKV order (reference gguf/models/{bloom,falcon,mpt}.py), then the
    native generic decoder (k-quant blocks kept for q4_k)"""
    import transformers as T
    from ipex_llm_amd.convert_model import export_gguf
    from ipex_llm_amd.gguf.api import load_gguf_model
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    torch.manual_seed(0)
    ref = T.AutoModelForCausalLM.from_config(_family(kind)).eval()
    f = export_gguf(ref, str(tmp_path / f"{kind}-{qt}.gguf"), qt)
    assert G.GGUFReader(f).architecture == ("falcon" if kind.startswith("falcon") else kind)
    dense, _ = load_gguf_model(f, dtype=torch.float32)
    ids = torch.randint(0, 256, (1, 9))
    with torch.no_grad():
        a, b = ref(ids).logits, dense(ids).logits
    assert ((a - b).norm() / a.norm()).item() < (1e-3 if qt == "f16" else 0.15)
    m, _ = AutoModelForCausalLM.from_gguf(f, low_bit="sym_int8", torch_dtype=torch.float32)
    assert getattr(m, "_illm_native_attached", False)
    with torch.no_grad():
        c = m(ids).logits.float()
    assert ((c - b).norm() / b.norm()).item() < 3e-2


def test_llm_convert_family_kquant(tmp_path):
    """llm_convert of a non-llama family (bloom) straight to a q4_k_m GGUF"""
    import transformers as T
    from ipex_llm_amd.convert_model import llm_convert
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    torch.manual_seed(0)
    ref = T.AutoModelForCausalLM.from_config(T.BloomConfig(vocab_size=256, hidden_size=256, n_layer=2,
                                                            n_head=4)).eval()
    p = str(tmp_path / "hf")
    ref.save_pretrained(p)
    f = llm_convert(p, str(tmp_path / "b.gguf"), "gguf_q4_k_m", model_family="bloom")
    assert G.GGUFReader(f).architecture == "bloom"
    m, _ = AutoModelForCausalLM.from_gguf(f, torch_dtype=torch.float32)
    ids = torch.randint(0, 256, (1, 8))
    with torch.no_grad():
        a, b = ref(ids).logits, m(ids).logits.float()
    assert ((a - b).norm() / a.norm()).item() < 0.15
