"""Bit-level parity helpers shared by the GPU tests (test infrastructure).

PCL writes std::numeric_limits<float>::quiet_NaN() (0x7FC00000) for points without a normal and
for descriptor rows it cannot compute; the product writes the same bits, so outputs are compared
as raw 32-bit patterns with NaN rows included (a NaN with another payload is a mismatch)."""
import numpy as np


def bits(a):
    return np.ascontiguousarray(np.asarray(a, np.float32)).view(np.uint32)


def bits_equal(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(bits(a), bits(b))
