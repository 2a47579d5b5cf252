"""C-ABI surface and host logic, no GPU: the library loads, exports every symbol declared in
include/tts_mi355x.h, validates configurations with the documented status codes, and the
Python drop-ins accept reference state_dicts and fail loudly off-device."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from _util import GOLDEN, hifigan_ctor
from oracle import glow_ref, hifigan_ref
from tts_amd import _native as N
from tts_amd import synthetic
from tts_amd.config import HIFIGAN_V1
from tts_amd.tts import Decoder
from tts_amd.vocoder import GAN, HifiganGenerator, setup_generator

HEADER = os.path.join(os.path.dirname(GOLDEN), "..", "include", "tts_mi355x.h")
V1 = dict(in_channels=80, out_channels=1, **HIFIGAN_V1)


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tts_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = N.lib()
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"{n} not exported"
        assert n in N.SIGNATURES, f"{n} has no ctypes signature"
    assert set(N.SIGNATURES) == set(names)


def test_version_and_target():
    assert N.lib().tts_abi_version() == N.ABI_VERSION == 115
    assert N.lib().tts_build_target() == b"gfx950"
    assert N.lib().tts_last_error() == b""


def test_library_built_from_these_sources():
    """Provenance: the loaded .so carries the hash of the sources in this tree (a stale or foreign
    build fails here, before any GPU run uses it)."""
    info = N.build_info()
    assert info["target"] == "gfx950"
    assert info["defs"] == "none", f"the in-tree library is a variant build ({info['defs']})"
    assert info["src"] == N.source_hash(), (
        f"libtts_mi355x.so was built from other sources (src={info['src']}, tree={N.source_hash()}): "
        "rebuild with make -C tts-3_amd")
    assert len(info["lib_sha256"]) == 16


def _cfg(**over):
    g = HifiganGenerator(**{**V1, **over})
    return g._cfg


def test_hifigan_weight_inventory_matches_module():
    g = HifiganGenerator(**V1)
    ws = g._weight_list()
    n = N.lib().tts_hifigan_num_weights(ctypes.byref(g._cfg))
    assert n == len(ws) == 2 + 8 + 4 * 3 * 12 + 2
    for i, w in enumerate(ws):
        assert N.lib().tts_hifigan_weight_numel(ctypes.byref(g._cfg), i) == w.size
    assert N.lib().tts_hifigan_weight_numel(ctypes.byref(g._cfg), n) == -1
    assert sum(w.size for w in ws) == 13926017  # HiFiGAN-v1 after weight-norm removal


@pytest.mark.parametrize(
    "over,code,msg",
    [
        (dict(upsample_kernel_sizes=[16, 15, 4, 4]), N.TTS_ERR_UNSUPPORTED, "2*factor"),
        (dict(upsample_factors=[8, 8, 3, 2], upsample_kernel_sizes=[16, 16, 6, 4]), N.TTS_ERR_UNSUPPORTED, "2, 4 or 8"),
        (dict(resblock_kernel_sizes=[3, 9, 11]), N.TTS_ERR_UNSUPPORTED, "kernel size"),
        (dict(resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 40]]), N.TTS_ERR_UNSUPPORTED, "dilation"),
    ],
)
def test_hifigan_config_validation(over, code, msg):
    with pytest.raises(N.NativeError) as e:
        HifiganGenerator(**{**V1, **over})
    assert e.value.code == code
    assert msg in str(e.value)


def test_out_channels_unsupported_status():
    with pytest.raises(N.NativeError) as e:
        HifiganGenerator(**{**V1, "out_channels": 4})
    assert e.value.code == N.TTS_ERR_UNSUPPORTED


def test_state_dict_keys_match_reference_checkpoints():
    sd = synthetic.hifigan_state_dict(seed=1)  # the same dict make_goldens.py loads into the reference
    g = HifiganGenerator(**V1)
    g.load_state_dict(sd)  # strict
    assert list(g.state_dict().keys()) == list(sd.keys())


def test_fold_matches_reference_remove_weight_norm():
    sd = synthetic.hifigan_state_dict(seed=2)
    g = HifiganGenerator(**V1)
    g.load_state_dict(sd)
    before = g._weight_list()
    g.remove_weight_norm()
    after = g._weight_list()
    folded = hifigan_ref.fold_weight_norm(sd, torch.float32)
    assert np.array_equal(before[0], folded["conv_pre.weight"].numpy())
    for a, b in zip(before, after):
        assert np.array_equal(a, b)
    assert "conv_pre.weight" in g.state_dict()


def test_cpu_module_refuses_to_run():
    g = HifiganGenerator(**V1)
    with pytest.raises(RuntimeError, match="ROCm device"):
        g.inference(torch.zeros(1, 80, 4))


def test_setup_generator_and_gan_surface(tmp_path):
    cfg = {"generator_model": "hifigan_generator", "audio": {"num_mels": 80},
           "generator_model_params": dict(HIFIGAN_V1)}
    gan = GAN.init_from_config(cfg)
    assert isinstance(gan.model_g, HifiganGenerator)
    sd = synthetic.hifigan_state_dict(seed=5)
    path = tmp_path / "ckpt.pth"
    torch.save({"model": {"model_g." + k: v for k, v in sd.items()}}, path)
    gan.load_checkpoint(cfg, str(path), eval=True)
    assert gan.model_d is None
    w = gan.model_g._weight_list()
    assert np.array_equal(w[0], hifigan_ref.fold_weight_norm(sd, torch.float32)["conv_pre.weight"].numpy())
    with pytest.raises(NotImplementedError):
        setup_generator({**cfg, "generator_model": "melgan_generator"})


def test_setup_generator_selects_math_mode(monkeypatch):
    """The fp32-faithful fast mode is the drop-in default, and a config can pick another one
    without code edits (generator_model_params, a top-level field, or the environment)."""
    monkeypatch.delenv("TTS_MI355X_MATH_MODE", raising=False)
    cfg = {"generator_model": "hifigan_generator", "audio": {"num_mels": 80},
           "generator_model_params": dict(HIFIGAN_V1)}
    g = setup_generator(cfg)
    assert g.math_mode == "f16x3" and g._cfg.math_mode == N.MATH_MODES["f16x3"]
    assert GAN(cfg).model_g.math_mode == "f16x3"
    assert HifiganGenerator(**V1).math_mode == "f16x3"
    assert Decoder(80, 192, 5, 1, 12, 4).math_mode == "f16x3"
    g = setup_generator({**cfg, "generator_model_params": dict(HIFIGAN_V1, math_mode="fp32")})
    assert g.math_mode == "fp32" and g._cfg.math_mode == 0
    g = setup_generator({**cfg, "math_mode": "fp32x6"})
    assert g._cfg.math_mode == N.MATH_MODES["fp32x6"]
    monkeypatch.setenv("TTS_MI355X_MATH_MODE", "fp32")
    assert setup_generator(cfg)._cfg.math_mode == 0
    monkeypatch.setenv("TTS_MI355X_MATH_MODE", "bf16")  # lower precision: explicit only
    with pytest.raises(ValueError, match="not fp32-faithful"):
        setup_generator(cfg)
    monkeypatch.setenv("TTS_MI355X_MATH_MODE", "tf32")
    with pytest.raises(ValueError, match="TTS_MI355X_MATH_MODE"):
        HifiganGenerator(**V1)


def test_lib_refuses_other_abi_revision(monkeypatch):
    """lib() checks tts_abi_version() before binding: a library of another revision would take
    pointers where it expects sizes."""
    lib = N.lib()
    assert lib.tts_abi_version() == N.ABI_VERSION
    monkeypatch.setattr(N, "_lib", None)
    monkeypatch.setattr(N, "ABI_VERSION", N.ABI_VERSION + 1)
    with pytest.raises(RuntimeError, match="C-ABI"):
        N.lib()
    monkeypatch.setattr(N, "ABI_VERSION", N.ABI_VERSION - 1)
    assert N.lib() is not None


def test_hifigan_generator_load_checkpoint(tmp_path):
    sd = synthetic.hifigan_state_dict(seed=6)
    path = tmp_path / "g.pth"
    torch.save({"model": sd}, path)
    g = HifiganGenerator(**V1)
    g.load_checkpoint({}, str(path), eval=True)
    assert not g.training
    assert not any(".parametrizations." in k for k in g.state_dict())


def test_glow_decoder_surface():
    cfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=12,
               num_coupling_layers=4)
    d = Decoder(**cfg, dropout_p=0.05, num_splits=4, num_squeeze=2)
    sd = synthetic.glow_decoder_state_dict(seed=7)
    d.load_state_dict(sd)  # strict: reference key set
    d.eval()
    d.store_inverse()
    ws = d._weight_list()
    n = N.lib().tts_glow_decoder_num_weights(ctypes.byref(d._cfg))
    assert n == len(ws) == 12 * (6 + 4 * 4 + 2)  # invconv weight_inv and weight (ABI 112)
    for i, w in enumerate(ws):
        assert N.lib().tts_glow_decoder_weight_numel(ctypes.byref(d._cfg), i) == w.size
    # W^-1 identical to the oracle's (reference store_inverse semantics)
    winv = torch.inverse(d.flows[1].weight.detach().float())
    wf = sd["flows.1.weight"].float()
    assert torch.equal(winv, torch.inverse(wf.t().contiguous().t()))
    with pytest.raises(RuntimeError, match="ROCm device"):
        d(torch.zeros(1, 80, 8), torch.ones(1, 1, 8), reverse=True)
    with pytest.raises(RuntimeError, match="ROCm device"):
        d(torch.zeros(1, 80, 8), torch.ones(1, 1, 8), reverse=False)


def test_glow_decoder_speaker_surface():
    """c_in_channels > 0: the reference key set (every WN's cond_layer, weight-normed) loads strictly
    and the weight inventory lines up with the C-ABI's."""
    cfg = dict(in_channels=80, hidden_channels=192, kernel_size=5, dilation_rate=1, num_flow_blocks=3,
               num_coupling_layers=4)
    d = Decoder(**cfg, num_splits=4, num_squeeze=2, c_in_channels=24)
    sd = synthetic.glow_decoder_state_dict(**cfg, c_in_channels=24, seed=8)
    d.load_state_dict(sd)
    assert "flows.2.wn.cond_layer.parametrizations.weight.original1" in sd
    d.store_inverse()
    ws = d._weight_list()
    n = N.lib().tts_glow_decoder_num_weights(ctypes.byref(d._cfg))
    assert n == len(ws) == 3 * 26
    for i, w in enumerate(ws):
        assert N.lib().tts_glow_decoder_weight_numel(ctypes.byref(d._cfg), i) == w.size
    with pytest.raises(RuntimeError, match="ROCm device"):
        d(torch.zeros(1, 80, 8), torch.ones(1, 1, 8), g=torch.zeros(1, 24, 1), reverse=True)


def test_glow_config_validation():
    c = N.TtsGlowDecoderCfg(80, 192, 5, 1, 12, 4, 3, 2, 0, 0)
    assert N.lib().tts_glow_decoder_num_weights(ctypes.byref(c)) == -N.TTS_ERR_UNSUPPORTED
    assert b"num_splits" in N.lib().tts_last_error()
    c = N.TtsGlowDecoderCfg(80, 192, 5, 1, 12, 4, 4, 2, 0, 16)  # speaker-conditioned: + cond_layer w, b per flow
    assert N.lib().tts_glow_decoder_num_weights(ctypes.byref(c)) == 12 * 26
    c = N.TtsGlowDecoderCfg(80, 192, 5, 1, 12, 4, 4, 2, 0, -1)
    assert N.lib().tts_glow_decoder_num_weights(ctypes.byref(c)) == -N.TTS_ERR_INVALID
    c = N.TtsGlowDecoderCfg(80, 192, 5, 1, 12, 4, 4, 2, 0, 0, N.MATH_MODES["f16x3"])
    assert N.lib().tts_glow_decoder_num_weights(ctypes.byref(c)) == 12 * 24  # f16x3 accepted (24 tensors per flow)
    c = N.TtsGlowDecoderCfg(80, 192, 5, 1, 12, 4, 4, 2, 0, 0, 9)
    assert N.lib().tts_glow_decoder_num_weights(ctypes.byref(c)) == -N.TTS_ERR_INVALID


def test_math_modes_and_tile_tables():
    lib = N.lib()
    assert N.MATH_MODES == {"fp32": 0, "fp32x6": 1, "f16x3": 2, "bf16": 3}
    for m in N.MATH_MODES.values():
        assert lib.tts_op_conv1d_num_tiles(m) >= 3
    assert lib.tts_op_conv1d_num_tiles(7) == -N.TTS_ERR_INVALID
    g = HifiganGenerator(**V1, math_mode="f16x3")
    assert g._cfg.math_mode == 2


def test_null_arguments_return_invalid():
    lib = N.lib()
    assert lib.tts_hifigan_create(None, None, 0, None) == N.TTS_ERR_INVALID
    assert lib.tts_hifigan_forward(None, None, 1, 80, 4, 0, None, None, None) == N.TTS_ERR_INVALID
    assert b"NULL" in lib.tts_last_error()
    assert lib.tts_hifigan_destroy(None) == N.TTS_OK
    assert lib.tts_glow_decoder_destroy(None) == N.TTS_OK


# ------------------------------------------------------------------------ Glow-TTS encoder / glue
def _glow_tts_cfg(**over):
    from tts_amd.config import GLOW_TTS_ENCODER

    return dict(GLOW_TTS_ENCODER, num_chars=64, **over)


def test_glow_encoder_weight_inventory_matches_reference_state_dict():
    from tts_amd.tts import Encoder

    cfg = _glow_tts_cfg()
    sd = synthetic.glow_encoder_state_dict(**cfg, seed=1)
    e = Encoder(cfg["num_chars"], cfg["out_channels"], cfg["hidden_channels"], cfg["hidden_channels_dp"],
                cfg["encoder_type"], cfg["encoder_params"], mean_only=True, use_prenet=True)
    e.load_state_dict(sd)  # strict: the reference's key set
    ws = e._weight_list()
    n = N.lib().tts_glow_encoder_num_weights(ctypes.byref(e._cfg))
    assert n == len(ws) == 1 + 14 + 6 * 16 + 2 + 10
    for i, w in enumerate(ws):
        assert N.lib().tts_glow_encoder_weight_numel(ctypes.byref(e._cfg), i) == w.size
    assert sum(w.size for w in ws) == sum(v.numel() for v in sd.values())


def test_glow_encoder_rel_window_inventory():
    from tts_amd.tts import Encoder

    ep = {"kernel_size": 3, "dropout_p": 0.1, "num_layers": 2, "num_heads": 2, "hidden_channels_ffn": 192,
          "rel_attn_window_size": 4}
    sd = synthetic.glow_encoder_state_dict(num_chars=40, out_channels=24, hidden_channels=96, hidden_channels_dp=64,
                                           encoder_params=ep, mean_only=False, use_prenet=False, seed=2)
    e = Encoder(40, 24, 96, 64, "rel_pos_transformer", ep, mean_only=False, use_prenet=False)
    e.load_state_dict(sd)
    ws = e._weight_list()
    assert len(ws) == N.lib().tts_glow_encoder_num_weights(ctypes.byref(e._cfg))
    assert sum(w.size for w in ws) == sum(v.numel() for v in sd.values())


def test_glow_encoder_c_validation_codes():
    c = N.TtsGlowEncoderCfg(num_chars=10, out_channels=80, hidden_channels=192, hidden_channels_dp=256,
                            hidden_channels_ffn=768, num_heads=5, num_layers=6, kernel_size=3)
    assert N.lib().tts_glow_encoder_num_weights(ctypes.byref(c)) == -N.TTS_ERR_INVALID  # transformer.py:75
    assert b"num_heads" in N.lib().tts_last_error()
    c.num_heads = 2
    n0 = N.lib().tts_glow_encoder_num_weights(ctypes.byref(c))
    assert n0 > 0
    c.c_in_channels = 16  # speaker-conditioned duration predictor: same tensors, conv_1 [dp][H + 16][3]
    assert N.lib().tts_glow_encoder_num_weights(ctypes.byref(c)) == n0
    c.c_in_channels = -1
    assert N.lib().tts_glow_encoder_num_weights(ctypes.byref(c)) == -N.TTS_ERR_INVALID
    c.c_in_channels, c.math_mode = 0, N.MATH_MODES["f16x3"]
    assert N.lib().tts_glow_encoder_num_weights(ctypes.byref(c)) == -N.TTS_ERR_UNSUPPORTED


def test_glow_tts_multispeaker_surface():
    """init_multispeaker (glow_tts.py:107-135): use_speaker_embedding -> emb_g [num_speakers, H_enc] and
    c_in = H_enc; use_d_vector_file -> c_in = d_vector_dim (512 by default).  The reference key set loads
    strictly, the duration predictor's conv_1 takes H + c_in inputs, and _set_speaker_input's
    errors (:170-174) are raised before any device work."""
    from tts_amd.tts import GlowTTS

    m = GlowTTS(dict(num_chars=64, use_speaker_embedding=True, num_speakers=7))
    assert m.c_in_channels == 192 and m.encoder.c_in_channels == 192 and m.decoder.c_in_channels == 192
    assert list(m.state_dict())[0] == "emb_g.weight" and m.emb_g.weight.shape == (7, 192)
    ecfg = _glow_tts_cfg(c_in_channels=192)
    esd = synthetic.glow_encoder_state_dict(**ecfg, seed=3)
    assert esd["duration_predictor.conv_1.weight"].shape == (256, 384, 3)
    m.encoder.load_state_dict(esd)
    ws = m.encoder._weight_list()
    assert len(ws) == N.lib().tts_glow_encoder_num_weights(ctypes.byref(m.encoder._cfg))
    for i, w in enumerate(ws):
        assert N.lib().tts_glow_encoder_weight_numel(ctypes.byref(m.encoder._cfg), i) == w.size
    tok, lens = torch.zeros(2, 5, dtype=torch.int64), torch.tensor([5, 3])
    with pytest.raises(ValueError, match="together"):
        m.inference(tok, {"x_lengths": lens, "speaker_ids": torch.tensor([0, 1]), "d_vectors": torch.zeros(2, 192)})
    with pytest.raises(ValueError, match="speaker_ids or d_vectors"):
        m.inference(tok, {"x_lengths": lens})
    d = GlowTTS(dict(num_chars=64, use_d_vector_file=True))
    assert d.c_in_channels == 512 and not hasattr(d, "emb_g")
    assert GlowTTS(dict(num_chars=64, use_d_vector_file=True, d_vector_dim=256)).decoder.c_in_channels == 256
    with pytest.raises(ValueError, match="without enabling speaker embedding"):
        d.inference(tok, {"x_lengths": lens, "speaker_ids": torch.tensor([0, 1])})
    single = GlowTTS(dict(num_chars=64))
    with pytest.raises(ValueError, match="single-speaker"):
        single.inference(tok, {"x_lengths": lens, "d_vectors": torch.zeros(2, 64)})
    with pytest.raises(RuntimeError, match="ROCm device"):
        m.encoder(tok, lens, g=torch.zeros(2, 192, 1))


@pytest.mark.parametrize("over,code", [
    (dict(encoder_params={"kernel_size": 9, "num_layers": 1, "num_heads": 2, "hidden_channels_ffn": 8}),
     N.TTS_ERR_UNSUPPORTED),
])
def test_glow_encoder_config_validation(over, code):
    from tts_amd.tts import Encoder

    cfg = _glow_tts_cfg(**over)
    with pytest.raises(N.NativeError) as e:
        Encoder(cfg["num_chars"], cfg["out_channels"], cfg["hidden_channels"], cfg["hidden_channels_dp"],
                cfg["encoder_type"], cfg["encoder_params"], mean_only=True)
    assert e.value.code == code


ENC_TYPES = [
    ("gated_conv", {"kernel_size": 5, "dropout_p": 0.1, "num_layers": 9}, True, 1 + 9 * 4 + 4 + 10),
    ("residual_conv_bn", {"kernel_size": 4, "dilations": [1, 2, 4] * 4 + [1], "num_conv_blocks": 2,
                          "num_res_blocks": 13}, False, 1 + 13 * 2 * 6 + 6 + 4 + 10),
    ("time_depth_separable", {"kernel_size": 5, "num_layers": 9}, True, 1 + 14 + 9 * 18 + 4 + 10),
]


@pytest.mark.parametrize("et,ep,pre,nw", ENC_TYPES, ids=[t[0] for t in ENC_TYPES])
def test_glow_encoder_other_types_inventory(et, ep, pre, nw):
    """gated_conv / residual_conv_bn / time_depth_separable (encoder.py:112-127, the reference's
    suggested encoder_params :59-75): the reference's key set (BatchNorm buffers included) loads
    strictly, and every tensor handed to the C-ABI has the size it expects."""
    from tts_amd.tts import Encoder

    sd = synthetic.glow_encoder_state_dict(num_chars=40, out_channels=80, hidden_channels=192, hidden_channels_dp=256,
                                           encoder_type=et, encoder_params=ep, mean_only=False, use_prenet=pre, seed=5)
    e = Encoder(40, 80, 192, 256, et, ep, mean_only=False, use_prenet=pre)
    e.load_state_dict(sd)
    ws = e._weight_list()
    assert len(ws) == N.lib().tts_glow_encoder_num_weights(ctypes.byref(e._cfg)) == nw
    for i, w in enumerate(ws):
        assert N.lib().tts_glow_encoder_weight_numel(ctypes.byref(e._cfg), i) == w.size
    tracked = sum(v.numel() for k, v in sd.items() if k.endswith("num_batches_tracked"))
    assert sum(w.size for w in ws) == sum(v.numel() for v in sd.values()) - tracked


def test_glow_encoder_layernorm2_and_input_length_surface():
    """layer_norm_type "2" (LayerNorm2: gamma / beta [C], transformer.py:386-387) and input_length
    (block-limited attention, :148-150) reach the C-ABI configuration."""
    from tts_amd.tts import Encoder

    ep = {"kernel_size": 3, "dropout_p": 0.1, "num_layers": 2, "num_heads": 2, "hidden_channels_ffn": 128,
          "rel_attn_window_size": 4, "input_length": 0, "layer_norm_type": "2"}
    sd = synthetic.glow_encoder_state_dict(num_chars=30, out_channels=16, hidden_channels=64, hidden_channels_dp=48,
                                           encoder_params=ep, mean_only=False, use_prenet=True, seed=4)
    assert sd["encoder.norm_layers_1.0.gamma"].shape == (64,)
    e = Encoder(30, 16, 64, 48, "rel_pos_transformer", ep, mean_only=False, use_prenet=True)
    e.load_state_dict(sd)
    assert (e._cfg.layer_norm_type, e._cfg.has_input_length, e._cfg.input_length) == (2, 1, 0)
    ws = e._weight_list()
    assert len(ws) == N.lib().tts_glow_encoder_num_weights(ctypes.byref(e._cfg))
    for i, w in enumerate(ws):
        assert N.lib().tts_glow_encoder_weight_numel(ctypes.byref(e._cfg), i) == w.size
    with pytest.raises(ValueError, match="Unknown layer norm type"):
        Encoder(30, 16, 64, 48, "rel_pos_transformer", dict(ep, layer_norm_type="3"))


def test_glow_encoder_types_and_cpu_raise():
    from tts_amd.tts import Encoder, GlowTTS

    with pytest.raises(ValueError, match="Unkown encoder type"):  # encoder.py:123, sic
        Encoder(10, 80, 192, 256, "conformer", {})
    # the reference calls residual_conv_bn's nn.Sequential prenet with (x, x_mask): TypeError in forward
    e = Encoder(10, 80, 64, 48, "residual_conv_bn", {"kernel_size": 4, "dilations": [1], "num_conv_blocks": 2,
                                                     "num_res_blocks": 1}, use_prenet=True)
    with pytest.raises(TypeError):
        e(torch.zeros(1, 8, dtype=torch.long), torch.tensor([8]))
    c = N.TtsGlowEncoderCfg(num_chars=10, out_channels=80, hidden_channels=64, hidden_channels_dp=48,
                            encoder_type=N.ENCODER_TYPES["residual_conv_bn"], kernel_size=4, num_conv_blocks=2,
                            num_res_blocks=1)
    c.dilations[0] = 9  # beyond the conv kernels' halo
    assert N.lib().tts_glow_encoder_num_weights(ctypes.byref(c)) == -N.TTS_ERR_UNSUPPORTED
    c.dilations[0], c.encoder_type = 1, 7
    assert N.lib().tts_glow_encoder_num_weights(ctypes.byref(c)) == -N.TTS_ERR_INVALID
    m = GlowTTS(dict(num_chars=32))
    with pytest.raises(RuntimeError, match="ROCm"):
        m.inference(torch.zeros(1, 4, dtype=torch.long), {"x_lengths": torch.tensor([4])})


def test_glow_tts_config_defaults_follow_reference():
    from tts_amd.tts import GlowTTS

    m = GlowTTS(dict(num_chars=32))
    assert m.inference_noise_scale == 0.0 and m.length_scale == 1.0  # glow_tts_config.py:151-152
    assert m.encoder.hidden_channels == 192 and m.encoder.hidden_channels_dp == 256
    assert m.decoder.num_flow_blocks == 12 and m.decoder.hidden_channels == 192
    keys = set(m.state_dict())
    assert "encoder.encoder.attn_layers.5.conv_o.weight" in keys
    assert "decoder.flows.35.wn.res_skip_layers.3.parametrizations.weight.original1" in keys


def test_xtts_generator_inventory_and_validation():
    cfg = dict(in_channels=1024, out_channels=1, resblock_type="1",
               resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], resblock_kernel_sizes=[3, 7, 11],
               upsample_kernel_sizes=[16, 16, 4, 4], upsample_initial_channel=512, upsample_factors=[8, 8, 2, 2],
               inference_padding=0, cond_channels=512, conv_pre_weight_norm=False, conv_post_weight_norm=False,
               conv_post_bias=False)
    g = HifiganGenerator(**cfg, cond_in_each_up_layer=True)
    sd = synthetic.hifigan_state_dict(**cfg, cond_in_each_up_layer=True, seed=1)
    g.load_state_dict(sd)  # strict: conds.* keys as the XTTS module
    ws = g._weight_list()
    assert len(ws) == N.lib().tts_hifigan_num_weights(ctypes.byref(g._cfg)) == 2 + 8 + 144 + 1 + 2 + 8
    for i, w in enumerate(ws):
        assert N.lib().tts_hifigan_weight_numel(ctypes.byref(g._cfg), i) == w.size
    with pytest.raises(N.NativeError):
        HifiganGenerator(**dict(cfg, cond_channels=0), cond_in_each_up_layer=True)


def test_vits_text_weight_inventories_match_modules():
    """TextEncoder / StochasticDurationPredictor: the tensors the drop-ins hand over (reference
    state_dict order) match the C-ABI inventory element by element; unsupported configurations are
    rejected with the documented codes (no GPU needed)."""
    from tts_amd.config import VITS_SDP, VITS_TEXT_ENCODER
    from tts_amd.tts import StochasticDurationPredictor, TextEncoder

    te = TextEncoder(64, 192, 192, 768, 2, 6, 3, 0.1)
    te.load_state_dict(synthetic.vits_text_encoder_state_dict(num_chars=64, **VITS_TEXT_ENCODER))
    ws = te._weight_list()
    assert len(ws) == N.lib().tts_vits_text_encoder_num_weights(ctypes.byref(te._cfg))
    for i, w in enumerate(ws):
        assert w.size == N.lib().tts_vits_text_encoder_weight_numel(ctypes.byref(te._cfg), i), i
    for gin in (0, 16):
        sdp = StochasticDurationPredictor(192, 192, 3, 0.5, 4, cond_channels=gin)
        sdp.load_state_dict(synthetic.vits_sdp_state_dict(**VITS_SDP, cond_channels=gin))
        ws = sdp._weight_list()
        assert len(ws) == N.lib().tts_vits_sdp_num_weights(ctypes.byref(sdp._cfg))
        for i, w in enumerate(ws):
            assert w.size == N.lib().tts_vits_sdp_weight_numel(ctypes.byref(sdp._cfg), i), i
    c = N.TtsVitsSdpCfg(192, 192, 3, 4, 0, 0, N.MATH_MODES["f16x3"])
    assert N.lib().tts_vits_sdp_num_weights(ctypes.byref(c)) == -N.TTS_ERR_UNSUPPORTED
    # language embeddings (ABI 115): the text encoder at H + L, the SDP's cond_lang
    te = TextEncoder(64, 192, 192, 768, 2, 6, 3, 0.1, language_emb_dim=4)
    ws = te._weight_list()
    assert ws[0].size == 64 * 192 and ws[1].size == 196 * 196  # emb at H, the transformer at H + L
    assert len(ws) == N.lib().tts_vits_text_encoder_num_weights(ctypes.byref(te._cfg))
    for i, w in enumerate(ws):
        assert w.size == N.lib().tts_vits_text_encoder_weight_numel(ctypes.byref(te._cfg), i), i
    for gin, L in ((0, 4), (16, 4)):
        sdp = StochasticDurationPredictor(192, 192, 3, 0.5, 4, cond_channels=gin, language_emb_dim=L)
        ws = sdp._weight_list()
        assert len(ws) == N.lib().tts_vits_sdp_num_weights(ctypes.byref(sdp._cfg))
        for i, w in enumerate(ws):
            assert w.size == N.lib().tts_vits_sdp_weight_numel(ctypes.byref(sdp._cfg), i), i
    # the deterministic duration predictor (use_sdp=False), every conditioning combination
    from tts_amd.tts import DurationPredictor

    for gin, L in ((0, 0), (16, 0), (0, 4), (16, 4)):
        dp = DurationPredictor(192, 256, 3, 0.5, cond_channels=gin, language_emb_dim=L)
        ws = dp._weight_list()
        assert len(ws) == N.lib().tts_vits_dp_num_weights(ctypes.byref(dp._cfg)) == 10 + 2 * bool(gin) + 2 * bool(L)
        for i, w in enumerate(ws):
            assert w.size == N.lib().tts_vits_dp_weight_numel(ctypes.byref(dp._cfg), i), i
    c = N.TtsVitsDpCfg(192, 256, 3, 0, 0, N.MATH_MODES["f16x3"])
    assert N.lib().tts_vits_dp_num_weights(ctypes.byref(c)) == -N.TTS_ERR_UNSUPPORTED
    c = N.TtsVitsDpCfg(192, 256, 4, 0, 0, N.MATH_MODES["fp32"])  # even kernel
    assert N.lib().tts_vits_dp_num_weights(ctypes.byref(c)) == -N.TTS_ERR_UNSUPPORTED
    t = N.TtsVitsTextEncoderCfg(64, 192, 192, 768, 3, 6, 3, 0, 0)  # 192 % 3 == 0 but dk = 64: fine
    assert N.lib().tts_vits_text_encoder_num_weights(ctypes.byref(t)) > 0
    t = N.TtsVitsTextEncoderCfg(64, 192, 192, 768, 5, 6, 3, 0, 0)  # channels not divisible by heads
    assert N.lib().tts_vits_text_encoder_num_weights(ctypes.byref(t)) == -N.TTS_ERR_INVALID
