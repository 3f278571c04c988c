"""The oracle (CPU restatement) against the golden vectors generated from the reference.

These pin the oracle before it is trusted as the checker of the HIP path (build contract ③).
"""
import hashlib

import numpy as np
import pytest
import torch

import golden_inputs as gi
from oracle import edsam, dggm as dggm_o, ratio as ratio_o
from rgbd_amd import init as winit

CASES = gi.decomposition_cases()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("i", range(len(CASES)), ids=[c[0] for c in CASES])
def test_decomposition_bit_exact(golden, i):
    g1 = golden("g1_decompose")
    name, d3, r = CASES[i]
    assert str(g1["names"][i]) == name
    assert str(g1["input_sha"][i]) == sha(d3), "input regeneration drifted"
    grey = edsam.to_grayscale(d3)
    assert str(g1["grey_sha"][i]) == sha(grey)
    err = str(g1["error"][i])
    if err:
        with pytest.raises(ValueError):
            edsam.histogram(grey)
        return
    dec = edsam.decompose(d3, r)
    np.testing.assert_array_equal(dec["hist"], g1[f"{i}_hist"])
    np.testing.assert_array_equal(dec["edges"].view(np.uint32), g1[f"{i}_edges"].view(np.uint32))
    assert dec["n_modes"] == int(g1[f"{i}_n_modes"])
    np.testing.assert_array_equal(np.array(dec["centers"], np.float32).view(np.uint32),
                                  g1[f"{i}_centers"].view(np.uint32))
    wins = np.array([[float(a), float(b)] for a, b in dec["windows"]], np.float64).reshape(-1, 2)
    np.testing.assert_array_equal(wins, g1[f"{i}_windows"])
    np.testing.assert_array_equal(dec["code"], g1[f"{i}_code"])
    H, W = d3.shape[1:]
    for s, (oh, ow) in enumerate(gi.pool_sizes(H, W)):
        np.testing.assert_array_equal(edsam.pooled_codes(dec["code"], oh, ow), g1[f"{i}_pooled{s}"])


def test_edge_cases_cover_branches(golden):
    g1 = golden("g1_decompose")
    names = [str(n) for n in g1["names"]]
    nm = {n: (int(g1[f"{i}_n_modes"]) if not str(g1["error"][i]) else -1) for i, n in enumerate(names)}
    # 0, 1, 2 and 3 modes, and both reference error paths, are all exercised
    assert nm["no_peak"] == 0 and nm["const"] == 1 and nm["low_prominence"] == 2
    assert nm["plateau"] == 3 and nm["tied"] == 3
    assert nm["all_nan"] == -1 and nm["tiny_range"] == -1


def _dsam_params(prefix, cin, cout):
    w = lambda k, s: torch.from_numpy(winit.value_for(prefix + k, s))  # noqa: E731
    return dict(conv_w=torch.stack([w(f"conv_layers.{i}.weight", (cout, cin, 3, 3)) for i in range(4)]),
                conv_b=torch.stack([w(f"conv_layers.{i}.bias", (cout,)) for i in range(4)]),
                proj_w=w("rgb_projection.weight", (cout, cin, 3, 3)))


@pytest.mark.parametrize("tag,cin,cout", [("a", 8, 16), ("b", 16, 32)])
def test_dsam_forward(golden, tag, cin, cout):
    g2 = golden("g2_dsam")
    p = _dsam_params(f"g2.{tag}.", cin, cout)
    for ci, case_idx in enumerate(gi.G2_CASES):
        _, d3, r = CASES[case_idx]
        dec = edsam.decompose(d3, r)
        y = edsam.dsam_forward(torch.from_numpy(g2[f"{tag}_{ci}_x"]), dec["code"], dec["n_masks"], **p)
        np.testing.assert_allclose(y.numpy(), g2[f"{tag}_{ci}_y"], rtol=1e-5, atol=1e-5)


def test_dggm_forward(golden):
    g3 = golden("g3_dggm")
    chans = [4, 8, 16, 32]
    ws = [torch.from_numpy(winit.value_for(f"g3.depth_enhancement_layers.{i}.0.weight", (c, 3, 1, 1)))
          for i, c in enumerate(chans)]
    bs = [torch.from_numpy(winit.value_for(f"g3.depth_enhancement_layers.{i}.0.bias", (c,)))
          for i, c in enumerate(chans)]
    outs = dggm_o.dggm_forward([torch.from_numpy(g3[f"color{i}"]) for i in range(4)],
                               torch.from_numpy(g3["grad"]), torch.from_numpy(g3["mask"]), ws, bs)
    for i in range(4):
        np.testing.assert_allclose(outs[i].numpy(), g3[f"out{i}"], rtol=1e-6, atol=1e-6)


def ratio_params():
    from rgbd_amd import params as ratio_shapes
    pre = "model.pixel_level_module.ratio_predictor."
    return {k: torch.from_numpy(winit.value_for(pre + k, s)) for k, s in ratio_shapes.RATIO_SHAPES.items()}


@pytest.mark.slow
def test_ratio_predictor_eval(golden):
    g4 = golden("g4_ratio")
    pv = gi.pixel_values(4, 2, 240, 320)
    assert str(g4["input_sha"]) == sha(pv)
    r = ratio_o.ratio_forward(torch.from_numpy(pv[:, 3:6]), ratio_params(), training=False)
    np.testing.assert_allclose(r.numpy(), g4["ratio"], rtol=1e-5, atol=1e-6)
