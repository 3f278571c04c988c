"""Test-only: compare a training step's gradients with the reference's (tests/golden/g6_grads.npz).

Per grad-receiving parameter tensor the fixture holds the float64 norm and sum of the reference's
float32 gradient and sampled values at golden_inputs.sample_index positions.  The comparison
separates two classes:

* gradients that are zero in exact arithmetic — the decoder self-attention key biases
  (softmax over keys is invariant to a bias added to every key, so d loss / d b_k = 0): the
  reference's are float32 rounding noise, 1e-10 of the model's largest gradient rms.  For them
  only the magnitude is compared: ours must be as negligible (rms <= ZERO_FLOOR x the model's
  largest reference rms);
* every other tensor: the relative error of the norm, the relative L2 error of the sampled
  values and the largest sampled error in units of the tensor's rms."""
import numpy as np

ZERO_CLASS = 1e-8   # reference rms / largest reference rms below this: zero in exact arithmetic
ZERO_FLOOR = 1e-7   # ours must stay below this fraction of the largest reference rms


def compare_grads(grads, g6, names=None):
    """grads: {name: flat float64 numpy gradient}.  Returns the worst values of each measure
    and the tensors they occur in."""
    names = [str(n) for n in (g6["all_names"] if names is None else names)]
    rms = {n: float(g6[n + "|norm"]) / np.sqrt(grads[n].size) for n in names}
    top = max(rms.values())
    rep = {"norm_rel": (0.0, None), "sample_l2": (0.0, None), "sample_max_over_rms": (0.0, None),
           "zero_class": [], "zero_class_worst": 0.0}
    for n in names:
        g = grads[n]
        if rms[n] < ZERO_CLASS * top:
            rep["zero_class"].append(n)
            rep["zero_class_worst"] = max(rep["zero_class_worst"], float(np.sqrt(np.mean(g * g))) / top)
            continue
        ref_norm = float(g6[n + "|norm"])
        val, want = g[g6[n + "|idx"]], g6[n + "|val"].astype(np.float64)
        m = {"norm_rel": abs(np.linalg.norm(g) - ref_norm) / ref_norm,
             "sample_l2": float(np.linalg.norm(val - want) / max(np.linalg.norm(want), 1e-300)),
             "sample_max_over_rms": float(np.abs(val - want).max() / rms[n])}
        for k, v in m.items():
            if v > rep[k][0]:
                rep[k] = (v, n)
    return rep
