"""Diagnostic: check cmpc_wave.hip's block-sweep inverse and symv against numpy (GPU)."""
import ctypes
import sys
from pathlib import Path

import numpy as np

lib = ctypes.CDLL(str(Path(__file__).resolve().parent / (sys.argv[1] if len(sys.argv) > 1 else "libwave_unit.so")))
P = ctypes.POINTER(ctypes.c_float)
lib.wave_invert.argtypes = [P, ctypes.c_int, P, P, P]
rng = np.random.default_rng(0)
for n in (1, 4, 5, 16, 17, 63, 100, 115, 128, 129, 141, 150, 160, 161, 180, 192):
    A = rng.standard_normal((n, n))
    S = A @ A.T + n * np.eye(n) * 0.5
    S32 = np.zeros((192, 192), np.float32)
    S32[:n, :n] = S
    x = np.zeros(192, np.float32)
    x[:n] = rng.standard_normal(n)
    out = np.zeros((192, 192), np.float32)
    y = np.zeros(192, np.float32)
    rc = lib.wave_invert(S32.ctypes.data_as(P), n, out.ctypes.data_as(P), x.ctypes.data_as(P),
                         y.ctypes.data_as(P))
    inv = np.linalg.inv(S)
    e_inv = np.max(np.abs(out[:n, :n] - inv)) / np.max(np.abs(inv))
    e_y = np.max(np.abs(y[:n] - inv @ x[:n])) / np.max(np.abs(inv @ x[:n]))
    print(f"n={n:4d} rc={rc} inverse rel err {e_inv:.2e}  symv rel err {e_y:.2e}  "
          f"pad max {np.max(np.abs(y[n:])) if n < 192 else 0:.1e}")
    sys.stdout.flush()

# condensation vs tests/algo_spec.condense on fixture instances
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tests"))
import algo_spec
from parity_util import load_fixture, fixture_batch
U8 = ctypes.POINTER(ctypes.c_uint8)
IP = ctypes.POINTER(ctypes.c_int)
lib.wave_condense.argtypes = [P, P, ctypes.c_int, P, P, U8, P, IP, P, P, P, P]
pr = algo_spec.Params()
Q2 = (2 * pr.Q).astype(np.float32); R2 = (2 * pr.R).astype(np.float32)
for name in ("qp_cfg1.npz", "qp_cfg2.npz"):
    fb = fixture_batch(load_fixture(name))
    worst = 0.0
    for i in range(8):
        A = np.ascontiguousarray(fb["Ad"][i], np.float32); B = np.ascontiguousarray(fb["Bd"][i], np.float32)
        ct = np.ascontiguousarray(fb["contact"][i] != 0, np.uint8)
        st = ct.T.astype(bool)
        nf = 3 * int(st.sum())
        if nf > 128:
            continue
        out = np.zeros((128, 128), np.float32); nn = ctypes.c_int(0)
        dvec = rng.standard_normal(192).astype(np.float32)
        vin = np.zeros(192, np.float32); vin[:nf] = rng.standard_normal(nf) * 50
        gout = np.zeros(192, np.float32); Eout = np.zeros(192, np.float32)
        rc = lib.wave_condense(Q2.ctypes.data_as(P), R2.ctypes.data_as(P), 16, A.ctypes.data_as(P),
                               B.ctypes.data_as(P), ct.ctypes.data_as(U8), out.ctypes.data_as(P), ctypes.byref(nn),
                               dvec.ctypes.data_as(P), vin.ctypes.data_as(P), gout.ctypes.data_as(P),
                               Eout.ctypes.data_as(P))
        fidx = np.array([12 * k + 3 * l + a for k in range(16) for l in range(4) if st[k, l] for a in range(3)])
        u = np.zeros(192, np.float32); u[fidx] = vin[:nf]
        gref, Eref = algo_spec.gradient(A, B, dvec.reshape(16, 12), pr.Q, pr.R, u.reshape(16, 12))
        eg = np.max(np.abs(gout[:nf] - gref.reshape(-1)[fidx])) / np.max(np.abs(gref))
        eE = np.max(np.abs(Eout - Eref.reshape(-1))) / np.max(np.abs(Eref))
        if eg > 1e-5 or eE > 1e-5:
            print(name, i, "gradient rel err", eg, "E rel err", eE)
        Bt = [B[k][:, [3 * l + a for l in range(4) if st[k, l] for a in range(3)]] for k in range(16)]
        Rt = np.concatenate([R2[3 * l:3 * l + 3] / 2 for k in range(16) for l in range(4) if st[k, l]])
        H = algo_spec.condense(A, Bt, pr.Q, Rt, 0.0)
        e = np.max(np.abs(out[:nf, :nf] - H)) / np.max(np.abs(H))
        worst = max(worst, e)
        if e > 1e-5:
            bad = np.argwhere(np.abs(out[:nf, :nf] - H) > 1e-5 * np.max(np.abs(H)))
            print(name, i, "n", nf, nn.value, "rel err", e, "bad entries", len(bad), bad[:6].tolist())
    print(name, "condense worst rel err", worst, "(gradient checked)")

# ill-conditioned case: the condensed fixture Hessians with the polish shift (sigma = 1e-6)
print("--- polish-like conditioning: spectral radius of I - M H (refinement contraction)")
for name in ("qp_cfg1.npz", "qp_cfg2.npz"):
    fb = fixture_batch(load_fixture(name))
    for i in range(4):
        A = np.asarray(fb["Ad"][i], np.float32); B = np.asarray(fb["Bd"][i], np.float32)
        st = (fb["contact"][i] != 0).T
        nf = 3 * int(st.sum())
        if nf > 128:
            continue
        Bt = [B[k][:, [3 * l + a for l in range(4) if st[k, l] for a in range(3)]] for k in range(16)]
        Rt = np.concatenate([pr.R[3 * l:3 * l + 3] for k in range(16) for l in range(4) if st[k, l]])
        H = algo_spec.condense(A, Bt, pr.Q, Rt, 1e-6).astype(np.float64)
        S32 = np.zeros((192, 192), np.float32); S32[:nf, :nf] = H
        out = np.zeros((192, 192), np.float32); x = np.zeros(192, np.float32); y = np.zeros(192, np.float32)
        lib.wave_invert(S32.ctypes.data_as(P), nf, out.ctypes.data_as(P), x.ctypes.data_as(P), y.ctypes.data_as(P))
        Mi = out[:nf, :nf].astype(np.float64)
        rad = np.max(np.abs(np.linalg.eigvals(np.eye(nf) - Mi @ H)))
        # fp32 scalar sweep (the previous kernel's algorithm) for comparison
        d = 1 / np.sqrt(np.diag(H)); T = (H * d[:, None] * d[None, :]).astype(np.float32)
        for kk in range(nf):
            piv = T[kk, kk]; col = T[:, kk].copy(); col[kk] = piv - 1
            T = (T - np.outer(col, col) / piv).astype(np.float32); T[kk, kk] -= 2
        Ms = (-T * d[:, None] * d[None, :]).astype(np.float64)
        rad_s = np.max(np.abs(np.linalg.eigvals(np.eye(nf) - Ms @ H)))
        print(f"{name} {i} n={nf} cond={np.linalg.cond(H):.1e}  rho(I-MH) block={rad:.2e} scalar={rad_s:.2e}")
