"""VITS flow C-ABI surface without a GPU: weight inventory, validation status codes, the
reference state_dict layout, and the loud failure off-device."""
import ctypes

import pytest
import torch

from tts_amd import _native as N
from tts_amd import synthetic
from tts_amd.config import VITS_FLOW
from tts_amd.tts import ResidualCouplingBlocks


def _flow(**over):
    cfg = dict(VITS_FLOW, **over)
    return ResidualCouplingBlocks(cfg["channels"], cfg["hidden_channels"], cfg["kernel_size"], cfg["dilation_rate"],
                                  cfg["num_layers"], num_flows=cfg["num_flows"],
                                  cond_channels=cfg.get("cond_channels", 0), math_mode=cfg.get("math_mode", "fp32"))


@pytest.mark.parametrize("cond", [0, 8])
def test_weight_inventory_matches_module(cond):
    f = _flow(cond_channels=cond)
    f.load_state_dict(synthetic.vits_flow_state_dict(cond_channels=cond, seed=3))  # strict: reference keys
    ws = f._weight_list()
    n = N.lib().tts_vits_flow_num_weights(ctypes.byref(f._cfg))
    assert n == len(ws) == 4 * (2 + 4 * 2 + 4 * 2 + (2 if cond else 0) + 2)
    for i, w in enumerate(ws):
        assert N.lib().tts_vits_flow_weight_numel(ctypes.byref(f._cfg), i) == w.size
    assert N.lib().tts_vits_flow_weight_numel(ctypes.byref(f._cfg), n) == -1


def test_state_dict_order_matches_reference_layout():
    sd = synthetic.vits_flow_state_dict(cond_channels=8, seed=5)
    f = _flow(cond_channels=8)
    f.load_state_dict(sd)
    assert list(f.state_dict().keys()) == list(sd.keys())
    assert "flows.0.enc.cond_layer.parametrizations.weight.original0" in sd


def test_validation_status_codes():
    lib = N.lib()
    c = N.TtsVitsFlowCfg(191, 192, 5, 1, 4, 4, 0, 0)
    assert lib.tts_vits_flow_num_weights(ctypes.byref(c)) == -N.TTS_ERR_INVALID
    assert b"even" in lib.tts_last_error()
    c = N.TtsVitsFlowCfg(192, 192, 9, 1, 4, 4, 0, 0)
    assert lib.tts_vits_flow_num_weights(ctypes.byref(c)) == -N.TTS_ERR_UNSUPPORTED
    c = N.TtsVitsFlowCfg(192, 192, 5, 1, 4, 4, 0, N.MATH_MODES["f16x3"])  # f16x3: statistics per conv input
    assert lib.tts_vits_flow_num_weights(ctypes.byref(c)) > 0
    c = N.TtsVitsFlowCfg(192, 192, 5, 1, 4, 4, 0, 7)
    assert lib.tts_vits_flow_num_weights(ctypes.byref(c)) == -N.TTS_ERR_INVALID
    assert lib.tts_vits_flow_create(None, None, 0, None) == N.TTS_ERR_INVALID
    assert lib.tts_vits_flow_destroy(None) == N.TTS_OK


def test_cpu_module_refuses_to_run():
    f = _flow()
    with pytest.raises(RuntimeError, match="ROCm device"):
        f(torch.zeros(1, 192, 8), torch.ones(1, 1, 8), reverse=True)
    with pytest.raises(RuntimeError, match="ROCm device"):
        f(torch.zeros(1, 192, 8), torch.ones(1, 1, 8), reverse=False)


def test_posterior_encoder_surface():
    lib = N.lib()
    """PosteriorEncoder: the reference key set (networks.py:269-273, WN weight-normed) loads strictly,
    the weight inventory lines up with the C-ABI's, and the module refuses to run off-device."""
    from tts_amd import synthetic
    from tts_amd.tts import PosteriorEncoder

    for cond in (0, 8):
        pe = PosteriorEncoder(513, 192, 192, 5, 1, 16, cond_channels=cond)
        sd = synthetic.vits_posterior_state_dict(cond_channels=cond, seed=3)
        pe.load_state_dict(sd)  # strict
        assert list(pe.state_dict().keys()) == list(sd.keys())
        ws = pe._weight_list()
        n = lib.tts_vits_posterior_num_weights(ctypes.byref(pe._cfg))
        assert n == len(ws) == 2 + 4 * 16 + (2 if cond else 0) + 2
        for i, w in enumerate(ws):
            assert lib.tts_vits_posterior_weight_numel(ctypes.byref(pe._cfg), i) == w.size
        with pytest.raises(RuntimeError, match="ROCm device"):
            pe(torch.zeros(1, 513, 8), torch.tensor([8]))
    c = N.TtsVitsPosteriorCfg(513, 192, 192, 4, 1, 16, 0, 2)
    assert lib.tts_vits_posterior_num_weights(ctypes.byref(c)) == -N.TTS_ERR_UNSUPPORTED
    assert lib.tts_vits_posterior_create(None, None, 0, None) == N.TTS_ERR_INVALID
    assert lib.tts_vits_posterior_destroy(None) == N.TTS_OK
