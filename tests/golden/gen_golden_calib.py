"""Golden vectors for the Hessian calibration (main.py:296-308), written with torch exactly
as the reference driver does it: `activations.view(activations.size(2), -1)`, `.to(float64)`,
`a_aT = activations @ activations.T`, running sum, `activation_sum / (idx + 1)` after every
sample.  (main.py itself is not importable offline — it loads a HF model and dataset at
import time — so the four lines are replayed here on synthetic (1, T, D) activations.)

Run: python tests/golden/gen_golden_calib.py  -> tests/golden/calib_ref.npz"""
import os

import numpy as np
import torch

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "calib_ref.npz")


def main():
    g = torch.Generator().manual_seed(7)
    D = 96
    Ts = [5, 1, 17, 3]
    acts = [torch.randn(1, T, D, generator=g, dtype=torch.float32) * (0.5 + i) for i, T in enumerate(Ts)]
    activation_sum = None
    for idx, a in enumerate(acts):
        activations = a.view(a.size(2), -1)
        activations = activations.to(torch.float64)
        a_aT = torch.matmul(activations, activations.transpose(0, 1))
        if activation_sum is None:
            activation_sum = a_aT
        else:
            activation_sum += a_aT
        activation_sum = activation_sum / (idx + 1)
    np.savez_compressed(OUT, D=D, Ts=np.array(Ts), acts=np.concatenate([a.reshape(-1).numpy() for a in acts]),
                        H=activation_sum.numpy())


if __name__ == "__main__":
    main()
