"""numpy restatement of the CWT kernels' counter-based dropout draw (csrc/common.h
dropout_uniform / dropout_scale) for the dropout parity tests: splitmix64 finaliser of
(seed, stream, index), 24-bit uniform, keep iff u >= p, kept elements scaled by 1/(1-p)."""
import numpy as np

M64 = (1 << 64) - 1


def dropout_uniform(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        i = idx.astype(np.uint64)
        z = (np.uint64(seed & M64) + np.uint64(0x9E3779B97F4A7C15) * (i + np.uint64(1))
             + np.uint64((0xD1B54A32D192ED03 * (stream + 1)) & M64))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def dropout_scale(p: float, seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    u = dropout_uniform(seed, stream, idx)
    return np.where(u >= np.float32(p), np.float32(1.0) / np.float32(1.0 - p), np.float32(0.0)).astype(np.float32)
