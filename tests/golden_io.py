"""Load the committed golden vectors (tests/golden/*.npz, produced by make_golden.py)."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _bf16_bits_to_f32(u16):
    return (u16.astype(np.uint32) << 16).view(np.float32)


def load(name):
    """Return dict of arrays; bf16 payloads are decoded to float32 values (key without suffix)
    and their dtype is reported under '<key>__dt'."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    out = {}
    for k in z.files:
        a = z[k]
        if k.endswith("__bf16"):
            base = k[: -len("__bf16")]
            out[base] = _bf16_bits_to_f32(a)
            out[base + "__dt"] = "bfloat16"
        elif a.dtype == np.float16:
            out[k] = a.astype(np.float32)
            out[k + "__dt"] = "float16"
        elif a.dtype.kind == "f":
            out[k] = a
            out[k + "__dt"] = "float32"
        elif a.dtype.kind in "US":
            out[k] = str(a)
        else:
            out[k] = a.item() if a.ndim == 0 else a
    return out


def names(prefix):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def rel_err(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    t = np.complex128 if (np.iscomplexobj(a) or np.iscomplexobj(b)) else np.float64
    a, b = a.astype(t), b.astype(t)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
