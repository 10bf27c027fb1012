"""Encoder attention on the HIP flash kernel (csrc/hip/train_attn.hip forward,
training/flash_attn.py ``illm_flash``): bidirectional and causal, ragged
sequence lengths, against an fp32 PyTorch softmax attention; then BERT /
ViT / Whisper-encoder models converted with ``optimize_model`` (low-bit
linears + that attention) against the HF fp32 forward of the same random
weights (reference models/bert.py, whisper.py: optimized forward vs the
original, test_transformers_api_attention.py pattern)."""
import copy

import pytest
import torch
import transformers as T

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _ref_attn(q, k, v, causal):
    G = q.shape[1] // k.shape[1]
    k, v = k.repeat_interleave(G, 1).float(), v.repeat_interleave(G, 1).float()
    s = q.float() @ k.transpose(-1, -2) * q.shape[-1] ** -0.5
    if causal:
        T_ = q.shape[2]
        s = s.masked_fill(torch.ones(T_, T_, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    return (s.softmax(-1) @ v).transpose(1, 2)           # [B, T, H, D]


@pytest.mark.parametrize("T_", [1, 50, 77, 200, 1500])
@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [False, True])
def test_flash_forward_ragged(cuda, T_, D, causal):
    torch.manual_seed(T_ + D)
    q = torch.randn(2, 4, T_, D, device=cuda, dtype=torch.bfloat16)
    k = torch.randn(2, 2, T_, D, device=cuda, dtype=torch.bfloat16)
    v = torch.randn(2, 2, T_, D, device=cuda, dtype=torch.bfloat16)
    out, lse = torch.ops.ipex_llm_amd.train_attn_fwd(q, k, v, D ** -0.5, causal)
    assert out.shape == (2, T_, 4, D) and torch.isfinite(out.float()).all()
    assert _rel(out, _ref_attn(q, k, v, causal)) < 1e-2


def _count_flash(monkeypatch):
    from ipex_llm_amd.training import flash_attn
    n = [0]
    orig = flash_attn.flash_attention

    def counted(*a, **kw):
        n[0] += 1
        return orig(*a, **kw)
    monkeypatch.setattr(flash_attn, "flash_attention", counted)
    return n


def test_bert_encoder_flash(cuda, monkeypatch):
    from ipex_llm_amd import optimize_model
    torch.manual_seed(0)
    cfg = T.BertConfig(vocab_size=512, hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
                       intermediate_size=512, max_position_embeddings=256)
    ref = T.BertModel(cfg).eval()
    ids = torch.randint(0, 512, (2, 77))
    with torch.no_grad():
        want = ref(ids).last_hidden_state
    n = _count_flash(monkeypatch)
    m = optimize_model(copy.deepcopy(ref).to(torch.bfloat16), low_bit="bf16").to(cuda)
    with torch.no_grad():
        got = m(ids.to(cuda)).last_hidden_state
    assert n[0] == cfg.num_hidden_layers, n[0]
    assert _rel(got.cpu(), want) < 2e-2


def test_vit_encoder_flash(cuda, monkeypatch):
    from ipex_llm_amd import optimize_model
    torch.manual_seed(1)
    cfg = T.ViTConfig(hidden_size=256, num_hidden_layers=2, num_attention_heads=4, intermediate_size=512,
                      image_size=64, patch_size=8)
    ref = T.ViTModel(cfg).eval()
    px = torch.randn(2, 3, 64, 64)
    with torch.no_grad():
        want = ref(px).last_hidden_state                    # 65 tokens: ragged
    n = _count_flash(monkeypatch)
    m = optimize_model(copy.deepcopy(ref).to(torch.bfloat16), low_bit="bf16").to(cuda)
    with torch.no_grad():
        got = m(px.to(cuda, torch.bfloat16)).last_hidden_state
    assert n[0] == cfg.num_hidden_layers, n[0]
    assert _rel(got.float().cpu(), want) < 3e-2


def test_whisper_encoder_flash(cuda, monkeypatch):
    from ipex_llm_amd import optimize_model
    torch.manual_seed(2)
    cfg = T.WhisperConfig(vocab_size=512, d_model=256, encoder_layers=2, decoder_layers=2,
                          encoder_attention_heads=4, decoder_attention_heads=4, encoder_ffn_dim=512,
                          decoder_ffn_dim=512, num_mel_bins=80, max_source_positions=1500,
                          max_target_positions=64, pad_token_id=0, bos_token_id=1, eos_token_id=2,
                          decoder_start_token_id=3)
    ref = T.WhisperModel(cfg).eval()
    feats = torch.randn(1, 80, 3000)
    with torch.no_grad():
        want = ref.encoder(feats).last_hidden_state           # 1500 frames
    n = _count_flash(monkeypatch)
    m = optimize_model(copy.deepcopy(ref).to(torch.bfloat16), low_bit="bf16").to(cuda)
    with torch.no_grad():
        got = m.encoder(feats.to(cuda, torch.bfloat16)).last_hidden_state
    assert n[0] == cfg.encoder_layers, n[0]
    assert _rel(got.float().cpu(), want) < 3e-2


@pytest.mark.parametrize("fam", ["qwen2_audio", "llava"])
def test_multimodal_lowbit_on_gpu(cuda, fam):
    """audio / image + text models converted to sym_int8 run on the HIP low-bit
    GEMV/GEMM and match the fp32 CPU model"""
    from ipex_llm_amd import optimize_model
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    txt = dict(vocab_size=300, hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
               num_key_value_heads=2, max_position_embeddings=256)
    torch.manual_seed(0)
    ids = torch.randint(3, 280, (1, 24))
    if fam == "qwen2_audio":
        ac = dict(num_mel_bins=16, encoder_layers=2, encoder_attention_heads=4, encoder_ffn_dim=512, d_model=256,
                  max_source_positions=20)
        ref = T.Qwen2AudioForConditionalGeneration(
            T.Qwen2AudioConfig(audio_config=ac, text_config=txt, audio_token_index=290)).eval()
        ids[0, 1:11] = 290
        kw = dict(input_ids=ids, input_features=torch.randn(1, 16, 40), attention_mask=torch.ones_like(ids),
                  feature_attention_mask=torch.ones(1, 40, dtype=torch.long))
    else:
        vc = dict(model_type="clip_vision_model", hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
                  intermediate_size=512, image_size=56, patch_size=14, projection_dim=256)
        ref = T.LlavaForConditionalGeneration(
            T.LlavaConfig(vision_config=vc, text_config=dict(txt, model_type="llama"), image_token_index=290,
                          vision_feature_layer=-1)).eval()
        ids[0, 1:17] = 290
        kw = dict(input_ids=ids, pixel_values=torch.randn(1, 3, 56, 56))
    with torch.no_grad():
        want = ref(**kw).logits
    m = optimize_model(copy.deepcopy(ref).to(torch.bfloat16), low_bit="sym_int8").to(cuda)
    assert any(isinstance(x, LowBitLinear) and x.weight.is_cuda for x in m.modules())
    gkw = {k: (v.to(cuda, torch.bfloat16) if v.is_floating_point() else v.to(cuda)) for k, v in kw.items()}
    with torch.no_grad():
        got = m(**gkw).logits
    assert _rel(got.float().cpu(), want) < 5e-2
