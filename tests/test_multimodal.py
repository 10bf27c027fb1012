"""Non-decoder-only families on the HF forward over low-bit linears (the
reference optimises whisper, bert, qwen2_vl, mllama, minicpmv ... with
per-arch forwards; here they run the HF forward, the linears low-bit):
encoder-decoder speech (Whisper), encoders (BERT) and vision-language
(Qwen2-VL) load through the AutoModel classes and stay close to the dense
model.  Tiny random configs, CPU."""
import pytest
import torch


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def test_whisper_speech_seq2seq_lowbit(tmp_path):
    from transformers import WhisperConfig, WhisperForConditionalGeneration
    from ipex_llm_amd.transformers import AutoModelForSpeechSeq2Seq
    cfg = WhisperConfig(vocab_size=256, d_model=64, encoder_layers=2, decoder_layers=2, encoder_attention_heads=4,
                        decoder_attention_heads=4, encoder_ffn_dim=128, decoder_ffn_dim=128, num_mel_bins=16,
                        max_source_positions=32, max_target_positions=64, decoder_start_token_id=1, pad_token_id=0,
                        eos_token_id=2, bos_token_id=1)
    torch.manual_seed(0)
    ref = WhisperForConditionalGeneration(cfg).eval()
    p = str(tmp_path / "w")
    ref.save_pretrained(p)
    feats = torch.randn(1, 16, 64)
    dec = torch.tensor([[1, 5, 9, 11]])
    with torch.no_grad():
        want = ref(input_features=feats, decoder_input_ids=dec).logits
    m = AutoModelForSpeechSeq2Seq.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    with torch.no_grad():
        got = m(input_features=feats, decoder_input_ids=dec).logits
    assert _rel(got, want) < 5e-2
    out = m.generate(input_features=feats, max_new_tokens=4, min_new_tokens=4, do_sample=False)
    assert out.shape[1] >= 4


def test_bert_encoder_lowbit(tmp_path):
    from transformers import BertConfig, BertModel
    from ipex_llm_amd.transformers import AutoModel
    cfg = BertConfig(vocab_size=256, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                     intermediate_size=128, max_position_embeddings=64)
    torch.manual_seed(0)
    ref = BertModel(cfg).eval()
    p = str(tmp_path / "b")
    ref.save_pretrained(p)
    ids = torch.randint(3, 256, (2, 12))
    with torch.no_grad():
        want = ref(ids).last_hidden_state
    m = AutoModel.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    with torch.no_grad():
        got = m(ids).last_hidden_state
    assert _rel(got, want) < 5e-2


def test_qwen2_vl_image_text_lowbit(tmp_path):
    from transformers import Qwen2VLConfig, Qwen2VLForConditionalGeneration
    from ipex_llm_amd.transformers import AutoModelForImageTextToText, AutoModelForVision2Seq
    assert AutoModelForVision2Seq is AutoModelForImageTextToText
    text = dict(vocab_size=256, hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                num_key_value_heads=2, max_position_embeddings=256,
                rope_scaling={"type": "mrope", "mrope_section": [2, 3, 3]})
    vision = dict(depth=2, embed_dim=32, hidden_size=64, num_heads=4, mlp_ratio=2, patch_size=14,
                  spatial_merge_size=2, temporal_patch_size=2, in_channels=3)
    try:
        cfg = Qwen2VLConfig(text_config=text, vision_config=vision, image_token_id=250, video_token_id=251,
                            vision_start_token_id=252)
    except TypeError as e:                          # pragma: no cover - config layout of other versions
        pytest.skip(f"Qwen2VLConfig layout: {e}")
    torch.manual_seed(0)
    ref = Qwen2VLForConditionalGeneration(cfg).eval()
    p = str(tmp_path / "vl")
    ref.save_pretrained(p)
    ids = torch.randint(3, 240, (1, 10))
    with torch.no_grad():
        want = ref(input_ids=ids).logits
    m = AutoModelForImageTextToText.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    with torch.no_grad():
        got = m(input_ids=ids).logits
    assert _rel(got, want) < 5e-2
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    assert any(isinstance(x, LowBitLinear) for x in m.modules())


def test_mllama_image_text_lowbit():
    """Llama-3.2-Vision layout: tiled vision encoder (local + global layers),
    gated cross-attention layers in the text model (reference models/mllama.py)"""
    import copy
    import transformers as T
    from ipex_llm_amd import optimize_model
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    vc = dict(hidden_size=64, num_hidden_layers=2, num_global_layers=1, attention_heads=4, intermediate_size=128,
              image_size=28, patch_size=14, max_num_tiles=2, vision_output_dim=128, intermediate_layers_indices=[0],
              supported_aspect_ratios=[[1, 1], [1, 2]])
    tc = dict(vocab_size=300, hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
              num_key_value_heads=2, cross_attention_layers=[1], max_position_embeddings=256, pad_token_id=0,
              bos_token_id=1, eos_token_id=2)
    cfg = T.MllamaConfig(vision_config=vc, text_config=tc, image_token_index=290)
    torch.manual_seed(0)
    ref = T.MllamaForConditionalGeneration(cfg).eval()
    with torch.no_grad():                   # open the cross-attention / MLP gates (zero at init)
        for n, p in ref.named_parameters():
            if "gate" in n and p.numel() == 1:
                p.fill_(0.7)
    ids = torch.randint(3, 280, (1, 10))
    ids[0, 1] = 290
    cam = torch.zeros(1, 10, 1, 2, dtype=torch.long)
    cam[:, 1:, 0, :] = 1
    kw = dict(input_ids=ids, pixel_values=torch.randn(1, 1, 2, 3, 28, 28), aspect_ratio_ids=torch.tensor([[2]]),
              aspect_ratio_mask=torch.tensor([[[1, 1]]]), cross_attention_mask=cam)
    with torch.no_grad():
        want = ref(**kw).logits
        m = optimize_model(copy.deepcopy(ref), low_bit="sym_int8")
        got = m(**kw).logits
    assert any(isinstance(x, LowBitLinear) for x in m.model.vision_model.modules())
    assert any(isinstance(x, LowBitLinear) for x in m.model.language_model.modules())
    assert _rel(got, want) < 5e-2
    # the image matters: a different image changes the text logits
    kw2 = dict(kw, pixel_values=torch.randn(1, 1, 2, 3, 28, 28))
    with torch.no_grad():
        assert _rel(m(**kw2).logits, got) > 1e-3


def test_internvl_image_text_lowbit():
    """InternVL layout: InternViT encoder + pixel-shuffle projector + LLM
    (reference models/internvl.py)"""
    import copy
    import transformers as T
    from ipex_llm_amd import optimize_model
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    vc = dict(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
              image_size=[28, 28], patch_size=[14, 14])
    tc = dict(model_type="qwen2", vocab_size=300, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
              num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256)
    try:
        cfg = T.InternVLConfig(vision_config=vc, text_config=tc, image_token_id=290, downsample_ratio=0.5)
        torch.manual_seed(0)
        ref = T.InternVLForConditionalGeneration(cfg).eval()
    except (TypeError, ValueError) as e:               # pragma: no cover - config layout of other versions
        pytest.skip(f"InternVLConfig layout: {e}")
    n_img = ((28 // 14) ** 2) // 4                     # pixel shuffle 0.5: tokens per image
    ids = torch.randint(3, 280, (1, 10))
    ids[0, 1:1 + n_img] = 290
    kw = dict(input_ids=ids, pixel_values=torch.randn(1, 3, 28, 28))
    with torch.no_grad():
        want = ref(**kw).logits
        m = optimize_model(copy.deepcopy(ref), low_bit="sym_int8")
        got = m(**kw).logits
    assert any(isinstance(x, LowBitLinear) for x in m.modules())
    assert _rel(got, want) < 5e-2


def _mm_parity(ref, kw, tol=5e-2):
    import copy
    from ipex_llm_amd import optimize_model
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    with torch.no_grad():
        want = ref(**kw).logits
        m = optimize_model(copy.deepcopy(ref), low_bit="sym_int8")
        got = m(**kw).logits
    assert sum(isinstance(x, LowBitLinear) for x in m.modules()) > 0
    assert _rel(got, want) < tol
    return m


_TXT = dict(vocab_size=300, hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
            num_key_value_heads=2, max_position_embeddings=256)


def test_qwen2_audio_lowbit():
    """Qwen2-Audio: Whisper-style audio encoder + pooled projector + Qwen2
    (reference serving/fastapi audio path, models/qwen2_audio)"""
    import transformers as T
    ac = dict(num_mel_bins=16, encoder_layers=2, encoder_attention_heads=4, encoder_ffn_dim=128, d_model=64,
              max_source_positions=20)
    torch.manual_seed(0)
    ref = T.Qwen2AudioForConditionalGeneration(
        T.Qwen2AudioConfig(audio_config=ac, text_config=_TXT, audio_token_index=290)).eval()
    ids = torch.randint(3, 280, (1, 16))
    ids[0, 1:11] = 290                                  # 40 frames -> 20 (conv) -> 10 (pool)
    kw = dict(input_ids=ids, input_features=torch.randn(1, 16, 40), attention_mask=torch.ones_like(ids),
              feature_attention_mask=torch.ones(1, 40, dtype=torch.long))
    m = _mm_parity(ref, kw)
    with torch.no_grad():                                # the audio matters
        assert _rel(m(**dict(kw, input_features=torch.randn(1, 16, 40))).logits, m(**kw).logits) > 1e-3


def test_gemma3_image_text_lowbit():
    """Gemma-3 vision: SigLIP tower + pooled projector; the tower's
    nn.MultiheadAttention projections stay dense (torch reads their weights)"""
    import transformers as T
    vc = dict(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128, image_size=28,
              patch_size=14)
    torch.manual_seed(0)
    ref = T.Gemma3ForConditionalGeneration(
        T.Gemma3Config(vision_config=vc, text_config=dict(_TXT, head_dim=16, sliding_window=64),
                       mm_tokens_per_image=4, image_token_index=290)).eval()
    ids = torch.randint(3, 280, (1, 12))
    ids[0, 1:5] = 290
    _mm_parity(ref, dict(input_ids=ids, pixel_values=torch.randn(1, 3, 28, 28), token_type_ids=(ids == 290).long()))


def test_llava_image_text_lowbit():
    import transformers as T
    vc = dict(model_type="clip_vision_model", hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
              intermediate_size=128, image_size=28, patch_size=14, projection_dim=64)
    torch.manual_seed(0)
    ref = T.LlavaForConditionalGeneration(
        T.LlavaConfig(vision_config=vc, text_config=dict(_TXT, model_type="llama"), image_token_index=290,
                      vision_feature_layer=-1)).eval()
    ids = torch.randint(3, 280, (1, 12))
    ids[0, 1:5] = 290
    _mm_parity(ref, dict(input_ids=ids, pixel_values=torch.randn(1, 3, 28, 28)))


def test_janus_image_understanding_lowbit():
    """Janus: SigLIP-style understanding encoder + aligner + Llama (reference
    models/janus.py); the VQ-VAE generation head is built but unused here"""
    import transformers as T
    vc = dict(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128, image_size=28,
              patch_size=14, projection_dim=64)
    vq = dict(embed_dim=8, num_embeddings=32, latent_channels=32, base_channels=32, channel_multiplier=[1, 1],
              num_res_blocks=1, num_patches=2, image_token_embed_dim=64, projection_dim=64)
    torch.manual_seed(0)
    ref = T.JanusForConditionalGeneration(
        T.JanusConfig(vision_config=vc, text_config=dict(_TXT, model_type="llama"), vq_config=vq,
                      image_token_id=290)).eval()
    ids = torch.randint(3, 280, (1, 12))
    ids[0, 1:5] = 290
    _mm_parity(ref, dict(input_ids=ids, pixel_values=torch.randn(1, 3, 28, 28)))


def test_qwen2_5_omni_thinker_audio_lowbit():
    """Qwen2.5-Omni thinker (reference models/qwen2_5_omni.py): audio encoder
    + M-RoPE Qwen2 text model, converted end to end"""
    import transformers as T
    ac = dict(num_mel_bins=16, encoder_layers=2, encoder_attention_heads=4, encoder_ffn_dim=128, d_model=64,
              max_source_positions=20, n_window=10, output_dim=64)
    vc = dict(depth=2, hidden_size=64, intermediate_size=128, num_heads=4, out_hidden_size=64, patch_size=14,
              spatial_merge_size=2, temporal_patch_size=2, fullatt_block_indexes=[1], window_size=56)
    t = dict(_TXT, rope_parameters={"rope_type": "default", "rope_theta": 10000.0, "mrope_section": [2, 3, 3]})
    try:
        cfg = T.Qwen2_5OmniThinkerConfig(audio_config=ac, vision_config=vc, text_config=t, audio_token_index=291,
                                         image_token_index=290, video_token_index=292, vision_start_token_id=293,
                                         audio_start_token_id=294, audio_end_token_id=295)
        torch.manual_seed(0)
        ref = T.Qwen2_5OmniThinkerForConditionalGeneration(cfg).eval()
    except (TypeError, ValueError, KeyError) as e:     # pragma: no cover - config layout of other versions
        pytest.skip(f"Qwen2.5-Omni config layout: {e}")
    ids = torch.randint(3, 280, (1, 16))
    ids[0, 1:6] = 291
    _mm_parity(ref, dict(input_ids=ids, input_features=torch.randn(1, 16, 40), attention_mask=torch.ones_like(ids),
                         feature_attention_mask=torch.ones(1, 40, dtype=torch.long)))
