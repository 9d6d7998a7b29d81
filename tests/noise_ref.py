"""Host restatement of the product's counter-based softfloor noise (tests only).

The reference draws softfloor's noise with ``torch.rand_like`` (train.py:22);
the product draws it in-kernel from a counter-based hash so a training step
is reproducible and needs no RNG state on the device.  This numpy version
is bit-identical to the device code (``pfsgnn_uniform`` in
``csrc/pfsgnn_common.h``) and lets the oracle receive the same uniforms.

    key = fmix64(seed ^ 0xD1B54A32D192ED03)
    u(e) = (fmix64(key + (e + 1) * 0x9E3779B97F4A7C15) >> 40) * 2^-24
"""
import numpy as np

M64 = (1 << 64) - 1


def fmix64_int(z):
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def uniform_numpy(seed, E):
    key = np.uint64(fmix64_int(int(seed) ^ 0xD1B54A32D192ED03))
    e = np.arange(1, E + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = key + e * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return ((z >> np.uint64(40)).astype(np.float64) * (2.0 ** -24)).astype(np.float32)
