"""Float32 emulation of C1's 65536-point transform (16 x 4096 four-step, kernels_fs16.hpp) with different twiddle
sources, against the float64 FFT and against numpy/scipy's float32 FFT (what the float32 oracle uses).

Question (round-2 verdict): does the device's 65536-point DHT round deeper than the float32 oracle because
its twiddles are products of LDS seeds (W^k, W^4k, W^8k; up to four chained complex products for W^15k)?

The emulation follows the device's structure: stage A = 16-point DFT (4 x 4 radix-4 butterflies) per column,
times W_65536^{n2 k1}; stage B = radix-16 Stockham passes of the 4096-point FFT with per-pass twiddles.
Twiddle sources: 'seed' (fp32-rounded seeds and the device's product chain), 'twotab' (hi/lo fp32 tables, one
product), 'exact' (each twiddle rounded from float64 once).  Metrics: plain relative error of the spectrum,
and the error of U = IDFT(DFT(r) / (C - lambda)) -- C1's preconditioner with Ct = 0, which weights the low
modes -- for two real rows packed as one complex line (as the device does).

Result (CPU, this script): spectrum 1.83e-7 (seed/seed) vs 1.53e-7 (exact/exact) vs scipy float32 1.51e-7;
U: 1.12e-7 (seed/seed), 1.03e-7 (exact/exact), scipy 1.05e-7.  Exact twiddles would gain <= 8 % on the
preconditioned quantity, so the seeds are not what separates the device from the float32 oracle at
C1.

usage: python scripts/fft16_twiddle_study.py
"""
import numpy as np
import scipy.fft as sf

f32, c64 = np.float32, np.complex64


def W(n, m):
    return np.exp(-2j * np.pi * np.asarray(m, dtype=np.float64) / n)


def cmul(a, b):
    ar, ai, br, bi = a.real.astype(f32), a.imag.astype(f32), b.real.astype(f32), b.imag.astype(f32)
    return ((ar * br - ai * bi).astype(f32) + 1j * (ar * bi + ai * br).astype(f32)).astype(c64)


def tw_set(n, k, R, mode):
    """twiddles W_n^{r k}, r = 0 .. R-1 (arrays over k)"""
    k = np.asarray(k)
    if mode == "exact":
        return [W(n, r * k).astype(c64) for r in range(R)]
    if mode == "twotab":
        out = []
        for r in range(R):
            m = (r * k) % n
            out.append(cmul(W(n, (m >> 8) << 8).astype(c64), W(n, m & 255).astype(c64)))
        return out
    w1, w4, w8 = W(n, k).astype(c64), W(n, 4 * k).astype(c64), W(n, 8 * k).astype(c64)   # fft_lds.hpp seeds
    w = [np.ones_like(w1)] + [None] * (R - 1)
    w[1] = w1
    if R > 2:
        w[2] = cmul(w1, w1)
        w[3] = cmul(w[2], w1)
    if R > 4:
        w[4], w[5], w[6], w[7] = w4, cmul(w4, w1), cmul(w4, w[2]), cmul(w4, w[3])
    if R > 8:
        w[8] = w8
        for r in range(1, 8):
            w[8 + r] = cmul(w8, w[r])
    return w


def dft4(a, b, c, d):
    t0, t1, t2, t3 = (a + c).astype(c64), (a - c).astype(c64), (b + d).astype(c64), (b - d).astype(c64)
    t3m = (t3.imag - 1j * t3.real).astype(c64)
    return (t0 + t2).astype(c64), (t1 + t3m).astype(c64), (t0 - t2).astype(c64), (t1 - t3m).astype(c64)


def dft16(v):   # 4 x 4 with the internal W_16 twiddles (fft_lds.hpp dft_any<C, 16>)
    v = [v[..., i].astype(c64) for i in range(16)]
    for n1 in range(4):
        v[n1], v[n1 + 4], v[n1 + 8], v[n1 + 12] = dft4(v[n1], v[n1 + 4], v[n1 + 8], v[n1 + 12])
    for n1 in range(1, 4):
        for k2 in range(1, 4):
            v[n1 + 4 * k2] = cmul(v[n1 + 4 * k2], np.full(1, W(16, n1 * k2)).astype(c64))
    out = [None] * 16
    for k2 in range(4):
        out[k2], out[k2 + 4], out[k2 + 8], out[k2 + 12] = dft4(v[4 * k2], v[4 * k2 + 1], v[4 * k2 + 2], v[4 * k2 + 3])
    return np.stack(out, -1)


def stockham(x, mode):
    n = x.shape[-1]
    LS = 1
    x = x.astype(c64)
    while LS < n:
        R, nR = 16, n // 16
        j = np.arange(nR)
        k = j % LS
        v = np.stack([x[..., j + r * nR] for r in range(R)], -1)
        if LS > 1:
            ws = tw_set(LS * R, k, R, mode)
            for r in range(1, R):
                v[..., r] = cmul(v[..., r], ws[r])
        v = dft16(v)
        y = np.empty_like(x)
        for r in range(R):
            y[..., (j - k) * R + k + r * LS] = v[..., r]
        x, LS = y, LS * R
    return x


def fs16(x, modeA, modeB):
    v = dft16(x.reshape(16, 4096).T.astype(c64))           # stage A over n1 -> [n2][k1]
    ws = tw_set(65536, np.arange(4096), 16, modeA)
    for k1 in range(1, 16):
        v[:, k1] = cmul(v[:, k1], ws[k1])
    return stockham(v.T, modeB).T.reshape(-1)              # stage B over n2; k = k1 + 16 k2


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def main():
    rng = np.random.default_rng(0)
    N = 65536
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    ref = np.fft.fft(x)
    print("spectrum: scipy float32 %.3e" % rel(sf.fft(x.astype(c64)), ref))
    for mA in ("seed", "twotab", "exact"):
        for mB in ("seed", "exact"):
            print("spectrum: stage A %-6s stage B %-6s %.3e" % (mA, mB, rel(fs16(x, mA, mB), ref)))
    dx = 2.0 / N
    k = np.arange(N)
    den = 1.0 + 2 * (1 - np.cos(2 * np.pi * k / N)) / dx ** 2   # C - lambda, C = 1, pow = 1, Ct = 0
    r = rng.standard_normal((2, N))
    z = r[0] + 1j * r[1]

    def row0(Zs):
        return (Zs + np.conj(Zs[(-k) % N])) / 2

    U0 = np.fft.ifft(row0(np.fft.fft(z)) / den).real
    print("U (Ct = 0): scipy float32 %.3e" % rel(np.fft.ifft(row0(sf.fft(z.astype(c64)).astype(complex)) / den).real, U0))
    for mA in ("seed", "twotab", "exact"):
        for mB in ("seed", "exact"):
            Zd = fs16(z, mA, mB).astype(complex)
            print("U (Ct = 0): stage A %-6s stage B %-6s %.3e" % (mA, mB, rel(np.fft.ifft(row0(Zd) / den).real, U0)))


if __name__ == "__main__":
    main()
