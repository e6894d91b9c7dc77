"""Search for RMSNorm rows whose float mean depends on the summation order
(tests/test_gpu_ops.py _RMS_ORDER_ROWS).

ggml_compute_forward_rms_norm_f32 (reference ggml.c:6060-6065) adds the float squares
x[i] * x[i] to a double in index order.  A row [a, b, t, t, ..., t] with a^2 + b^2 = S
putting S / K exactly on a float rounding midpoint, and t^2 below half an ulp of S, has an
index-order sum of exactly S (every t^2 rounds away: the float mean is the tie, rounded to
even), while the exactly rounded sum keeps the (K - 2) t^2 and rounds the other way.  The
search draws 12-bit a and b (exact squares) until both the mean and the final RMSNorm scale
1 / sqrtf(mean + 1e-6f) differ between the two sums.  Prints the (a, b, t) per K.

    python tests/golden/make_rms_order_rows.py
"""
import math
import random

import numpy as np

f32 = np.float32


def scale_of(s, k):
    mean = f32(s / k)
    return f32(f32(1.0) / np.sqrt(f32(mean + f32(1e-6)), dtype=f32)), mean


def search(k, seed=1, tries=200000):
    rnd = random.Random(seed)
    for _ in range(tries):
        ea = rnd.randint(-2, 4)
        a = f32(rnd.randint(2048, 4095) * 2.0 ** (ea - 11))
        b = f32(rnd.randint(2048, 4095) * 2.0 ** (ea - 12 - rnd.randint(0, 12)))
        s = float(a * a) + float(b * b)
        r = s / k
        f = f32(r)
        up = (float(f) + float(np.nextafter(f, f32(np.inf)))) / 2
        dn = (float(f) + float(np.nextafter(f, f32(-np.inf)))) / 2
        if r != up and r != dn:
            continue
        half_ulp = math.ulp(s) / 2
        t2 = 2.0 ** math.floor(math.log2(half_ulp))
        if t2 >= half_ulp:
            t2 /= 2
        t = math.sqrt(t2)
        if f32(t) * f32(t) != f32(t2):
            continue
        row = np.full(k, f32(t), f32)
        row[0], row[1] = a, b
        seq = 0.0
        for v in row:
            seq += float(f32(v) * f32(v))
        exact = math.fsum(float(f32(v) * f32(v)) for v in row)
        sc_s, m_s = scale_of(seq, k)
        sc_e, m_e = scale_of(exact, k)
        if m_s != m_e and sc_s != sc_e:
            return float(a), float(b), t
    return None


if __name__ == "__main__":
    for k in (256, 4096, 5120):
        print(k, search(k))
