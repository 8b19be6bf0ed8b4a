"""CPU-side checks of libnerfmi.so: it loads, exports every symbol include/nerfmi.h declares,
rejects bad arguments without touching a GPU, and its weight packer produces the layout the
MLP kernel assumes.  The last part replays the kernel's register dataflow (layout.h) in numpy
on the host-packed buffer and compares with the oracle's NeRF.forward."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO
from oracle import nerf_oracle as O
from nerfmi import _lib

HEADERS = [os.path.join(REPO, "include", h) for h in ("nerfmi.h", "nerfmi_train.h")]


def header_symbols():
    text = "".join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r"\b(nerf_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.EXPORTED), "ctypes signature table out of sync with include/*.h"
    assert lib.nerf_abi_version() == _lib.ABI_VERSION == 11


def test_bad_arguments_are_reported_not_launched():
    lib = _lib.load()
    rc = lib.nerf_composite(None, None, None, 10, 64, None, None, None, None)
    assert rc == 1 and b"null pointer" in lib.nerf_last_error()
    rc = lib.nerf_composite(None, None, None, 10, 5000, None, None, None, None)
    assert rc == 3
    rc = lib.nerf_sample_importance(None, None, None, None, 4, 300, 128, None, None, 0, None, None, None)
    assert rc == 3
    rc = lib.nerf_mlp_forward(None, None, None, None, 4, 2, None, None, None, None, 0, None)
    assert rc == 1 and b"N must be 1" in lib.nerf_last_error()
    assert lib.nerf_render_workspace_bytes(0, 64, 128) == 0 or lib.nerf_render_workspace_bytes(0, 64, 128) >= 0
    assert lib.nerf_render_workspace_bytes(-1, 64, 0) == 0

    # empty inputs are a no-op, not an error
    assert lib.nerf_composite(None, None, None, 0, 64, None, None, None, None) == 0
    # training entry points
    rc = lib.nerf_composite_backward(None, None, None, None, None, 4, 64, 1.0, None, None, None, None)
    assert rc == 1 and b"null pointer" in lib.nerf_last_error()
    assert lib.nerf_composite_backward(None, None, None, None, None, 4, 5000, 1.0, None, None, None, None) == 3
    assert lib.nerf_composite_backward_grad(None, None, None, None, None, 4, 64, None, None, None) == 1
    assert lib.nerf_composite_backward_grad(None, None, None, None, None, 4, 0, None, None, None) == 3
    assert lib.nerf_composite_backward_grad(None, None, None, None, None, 0, 64, None, None, None) == 0
    # a backward on a workspace no nerf_train_forward wrote is refused before any launch (it would
    # not know which arithmetic wrote the saves, nor whether mask rows exist)
    fake = ctypes.c_void_p(0x1000)
    grads = (ctypes.c_void_p * 24)(*([0x1000] * 24))
    ws_bytes = lib.nerf_train_workspace_bytes(4, 8)
    rc = lib.nerf_train_backward(fake, fake, fake, fake, 4, 8, None, 0, grads, None, fake, ctypes.c_void_p(0x2000),
                                 ws_bytes, None)
    assert rc == 1 and b"no nerf_train_forward" in lib.nerf_last_error()
    assert lib.nerf_adam(None, None, None, None, 8, 1e-3, .9, .999, 1e-8, 0, None) == 1   # step counts from 1
    assert lib.nerf_wgrad(None, 1, 4, None, 4, 4, 1, 8, None, None, 0, None, 0, None) == 1
    ws = lib.nerf_wgrad_workspace_bytes(5000, 256, 256)
    # the 256 x 256 path's 2048-sample chunks, halved (down to one 16-sample stage) while a short GEMM has
    # fewer than 128 of them: 5000 samples -> 32-sample chunks, 157 of them, x N x (K + bias column)
    clen = 2048
    while clen > 16 and -(-5000 // clen) < 128:
        clen //= 2
    assert clen == 32 and ws == -(-5000 // clen) * (256 * 257 + 4) * 4
    assert lib.nerf_wgrad_workspace_bytes(262144, 256, 256) == 128 * (256 * 257 + 4) * 4   # production size: 2048-sample chunks
    assert lib.nerf_train_workspace_bytes(4096, 64) > 4096 * 64 * (2400 + 2312) * 4
    assert lib.nerf_mlp_backward(None, None, None, None, None, None, None, None, 0, None, None) == 0
    # post effects
    assert lib.nerf_effect_workspace_bytes(0, 8) == 0
    assert lib.nerf_effect_workspace_bytes(800, 800) >= 256 + 2 * 800 * 800 * 4
    rc = lib.nerf_effect_fog(None, None, 1, 8, 8, 0.1, None, None, 0, None)
    assert rc == 1 and b"nerf_effect_fog" in lib.nerf_last_error()
    assert lib.nerf_frame_fog(None, None, 8, 8, 0.1, None, None, 0, None) == 1
    assert b"nerf_frame_fog" in lib.nerf_last_error()
    rc = lib.nerf_effect_fog(None, None, 0, 8, 8, 0.1, None, None, 0, None)      # depth stride < 1
    assert rc == 1
    rc = lib.nerf_effect_toon(None, None, 1, 8, 8, 0.0, 1.0, None, None, 0, None)   # levels must be > 0
    assert rc == 1 and b"levels" in lib.nerf_last_error()
    assert lib.nerf_depth_normalize(None, 0, None, None, 0, None) == 0            # empty: no-op
    assert lib.nerf_depth_normalize(None, 5, None, None, 0, None) == 1


def host_pack(state):
    lib = _lib.load()
    ts = [state[k].contiguous().float() for k in O.STATE_KEYS]
    arr = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
    out = np.empty(lib.nerf_packed_weights_floats(), dtype=np.float32)
    assert lib.nerf_pack_weights_host(arr, out.ctypes.data) == 0
    return out


# ---- restatement of csrc/layout.h for the emulator
PE_STEPS, ACT_STEPS = 32, 128


def frag_ntiles(m):
    return 4 if m == 8 else 8


def frag_ksteps(m):
    return PE_STEPS if m in (0, 9) else ACT_STEPS


def frag_offset(m):
    return sum(frag_ntiles(i) * frag_ksteps(i) * 64 for i in range(m))


def pe_feature(p, h):
    if p < 30:
        i, c = divmod(p, 3)
        return 3 + 6 * i + (3 if h else 0) + c
    if p == 30:
        return 1 if h else 0
    return -1 if h else 2


def act_feature(ks, h):
    t, g = divmod(ks, 16)
    return 32 * t + (g & 3) + 8 * (g >> 2) + 4 * h


def frag_matrix(packed, m):
    """W as the kernel sees it: [n][slot], slot = 2*ks + h (k-step ks, lane half h)."""
    nt, ks = frag_ntiles(m), frag_ksteps(m)
    blk = packed[frag_offset(m): frag_offset(m) + nt * ks * 64].reshape(nt, ks // 4, 2, 32, 4)
    # [nt][kq][h][n%32][j] -> [n][kq][j][h]
    return blk.transpose(0, 3, 1, 4, 2).reshape(nt * 32, ks * 2).astype(np.float64)


def test_packed_fragments_are_permuted_weights(ref_state):
    packed = host_pack(ref_state)
    W = {m: ref_state[f"pts_linears.{m}.weight"].numpy() for m in range(8)}
    for m in range(1, 8):
        Wp = frag_matrix(packed, m)
        cols = [act_feature(s // 2, s % 2) for s in range(2 * ACT_STEPS)]
        assert np.array_equal(Wp, W[m][:, cols]), m
    Wp = frag_matrix(packed, 0)
    for s in range(64):
        f = pe_feature(s // 2, s % 2)
        assert np.array_equal(Wp[:, s], W[0][:, f] if f >= 0 else np.zeros(256)), s
    Wp = frag_matrix(packed, 9)
    for s in range(64):
        f = pe_feature(s // 2, s % 2)
        assert np.array_equal(Wp[:, s], W[4][:, 256 + f] if f >= 0 else np.zeros(256)), s
    Wd = ref_state["dir_linear.weight"].numpy()
    cols = [act_feature(s // 2, s % 2) for s in range(2 * ACT_STEPS)]
    assert np.array_equal(frag_matrix(packed, 8), Wd[:, cols])


def emulate_forward(packed, x, d, app):
    """The kernel's dataflow (csrc/mlp.hip) in float64 on the packed buffer."""
    off_bias = frag_offset(10)
    off_sw = off_bias + 8 * 256
    off_sb = off_sw + 256
    off_db = off_sb + 4
    off_dwd = off_db + 128
    off_aw = off_dwd + 128 * 27
    off_ab = off_aw + 128 * 32
    off_rw = off_ab + 128
    off_rb = off_rw + 3 * 128
    p = packed.astype(np.float64)
    enc = O.positional_encoding(torch.from_numpy(x), 10).numpy().astype(np.float64)
    pe_slots = np.stack([enc[:, pe_feature(s // 2, s % 2)] if pe_feature(s // 2, s % 2) >= 0
                         else np.zeros(len(x)) for s in range(64)], 1)

    def act_slots(h):
        return h[:, [act_feature(s // 2, s % 2) for s in range(256)]]

    bias = p[off_bias: off_bias + 8 * 256].reshape(8, 256)
    h = np.maximum(pe_slots @ frag_matrix(packed, 0).T + bias[0], 0)
    for m in range(1, 8):
        pre = act_slots(h) @ frag_matrix(packed, m).T + bias[m]
        if m == 4:
            pre += pe_slots @ frag_matrix(packed, 9).T
        h = np.maximum(pre, 0)
    sigma = np.maximum(h @ p[off_sw: off_sw + 256] + p[off_sb], 0)
    encd = O.positional_encoding(torch.from_numpy(d), 4).numpy().astype(np.float64)
    dvec = p[off_db: off_db + 128] + encd @ p[off_dwd: off_dwd + 128 * 27].reshape(128, 27).T
    appf = np.zeros(128) if app is None else p[off_ab: off_ab + 128] + app.astype(np.float64) @ \
        p[off_aw: off_aw + 128 * 32].reshape(128, 32).T
    hd = np.maximum(act_slots(h) @ frag_matrix(packed, 8).T + dvec, 0) + appf
    rgb = 1 / (1 + np.exp(-(hd @ p[off_rw: off_rw + 384].reshape(3, 128).T + p[off_rb: off_rb + 3])))
    return rgb, sigma[:, None]


def test_emulated_kernel_matches_oracle(ref_state, app_vec):
    packed = host_pack(ref_state)
    torch.manual_seed(5)
    x = torch.randn(256, 3) * 2
    d = torch.nn.functional.normalize(torch.randn(256, 3), dim=-1)
    for app in (None, app_vec):
        rgb, sigma = emulate_forward(packed, x.numpy(), d.numpy(), None if app is None else app.numpy())
        rgb_o, sigma_o = O.nerf_forward(ref_state, x, d, app)
        np.testing.assert_allclose(rgb, rgb_o.numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(sigma, sigma_o.numpy(), rtol=1e-4, atol=1e-6)


# ---- the split-f16 ("f16x3") region of the packed buffer (layout.h, csrc/mlp16.hip)
def s16_layer_ks(L):
    return 4 if L == 0 else (20 if L == 4 else 16)


def s16_layer_groups(L):
    return 1 if L == 8 else 2


def s16_chunk0(L):
    return sum(s16_layer_groups(i) * s16_layer_ks(i) // 2 for i in range(L))


def s16_base():
    f32_floats = frag_offset(10) + 8 * 256 + 256 + 4 + 128 + 128 * 27 + 128 * 32 + 128 + 384 + 4
    return (f32_floats + 255) // 256 * 256


def s16_consts(packed):
    base = s16_base() + frag_offset(10)
    c = packed[base: base + 48].astype(np.float64)
    return {"s_w": c[0:9], "inv_w": c[9:18], "R": c[18:26], "B": c[26:34]}


def s16_source_col(m, ks, h, j):
    if m not in (0, 9):
        t, s = divmod(ks, 2)
        return 32 * t + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3)
    f = pe_feature(8 * ks + j, h)
    return f if f < 0 else (256 if m == 9 else 0) + f


def s16_layer_cols(L):
    """Natural input column of each k slot (k = 16 ks + 8 h + j) of layer L, or -1."""
    cols = []
    for ks in range(s16_layer_ks(L)):
        m = 8 if L == 8 else (9 if L == 4 and ks >= 16 else L)
        ksm = ks - 16 if m == 9 else ks
        cols += [s16_source_col(m, ksm, h, j) for h in range(2) for j in range(8)]
    return cols


def s16_layer(packed, L):
    """(hi, lo) of layer L as [n][k] in the kernel's k order, decoded from the chunk stream."""
    G, KS = s16_layer_groups(L), s16_layer_ks(L)
    off = s16_base() + s16_chunk0(L) * 4096
    raw = packed[off: off + G * KS // 2 * 4096].view(np.float16)
    raw = raw.reshape(G, KS // 2, 2, 4, 2, 2, 32, 8)          # g, i, kk, ti, part, h, n, j
    w = raw.transpose(4, 0, 3, 6, 1, 2, 5, 7).reshape(2, G * 128, KS * 16).astype(np.float64)
    return w[0], w[1]


def layer_weight(state, L):
    return (state["dir_linear.weight"] if L == 8 else state[f"pts_linears.{L}.weight"]).numpy().astype(np.float64)


def test_split_f16_stream_reconstructs_the_weights(ref_state):
    packed = host_pack(ref_state)
    c = s16_consts(packed)
    assert s16_chunk0(9) == 128
    assert np.all(c["s_w"] * c["inv_w"] == 1.0)
    for L in range(9):
        hi, lo = s16_layer(packed, L)
        W = layer_weight(ref_state, L)
        cols = s16_layer_cols(L)
        ref = np.stack([W[:, k] if k >= 0 else np.zeros(W.shape[0]) for k in cols], 1)
        mx = np.abs(ref).max()
        assert 2.0 ** 13 <= mx * c["s_w"][L] < 2.0 ** 14, L      # the scale puts the max just under 2^14
        assert np.array_equal(hi, (ref * c["s_w"][L]).astype(np.float32).astype(np.float16).astype(np.float64)), L
        assert np.abs((hi + lo) * c["inv_w"][L] - ref).max() <= mx * 2.0 ** -23, L
        if L < 8:
            Wfull = W if L != 8 else W[:, :256]
            l1 = np.abs(Wfull).sum(1).max()
            assert l1 <= c["R"][L] <= l1 * 1.001, L               # rigorous bound constant
            assert c["B"][L] == np.abs(ref_state[f"pts_linears.{L}.bias"].numpy()).max()


def emulate_forward_f16x3(packed, x, d, app):
    """csrc/mlp16.hip's dataflow on the host-packed buffer: per-sample power-of-two scales from the
    bound R max|a| + B, f16 hi/lo split in float32, the three products accumulated in float64."""
    c = s16_consts(packed)
    f32 = np.float32

    def split(v):
        v = v.astype(f32)
        hi = v.astype(np.float16)
        lo = (v - hi.astype(f32)).astype(np.float16)
        return hi.astype(np.float64), lo.astype(np.float64)

    def scale_of(bound):
        e = np.frexp(bound.astype(f32))[1]
        return np.ldexp(1.0, 14 - e)

    def dense(L, a_cols, s):
        hi, lo = s16_layer(packed, L)
        ah, al = split(a_cols * s[:, None])
        assert np.abs(ah).max() < 2.0 ** 15
        return (ah @ hi.T + al @ hi.T + ah @ lo.T) / (c["s_w"][L] * s)[:, None]

    enc = O.positional_encoding(torch.from_numpy(x), 10).numpy().astype(np.float64)
    m_pe = np.maximum(1.0, np.abs(x).max(1).astype(np.float64))
    bias = packed[frag_offset(10): frag_offset(10) + 8 * 256].reshape(8, 256).astype(np.float64)

    def inputs(L, h):
        full = np.concatenate([h, enc], 1) if L == 4 else (enc if L == 0 else h)
        return np.stack([full[:, k] if k >= 0 else np.zeros(len(x)) for k in s16_layer_cols(L)], 1)

    s = scale_of(m_pe)
    m_in = m_pe
    h = None
    for L in range(8):
        y = dense(L, inputs(L, h), s) + bias[L]
        bound = c["R"][L] * m_in + c["B"][L]
        h = np.maximum(y, 0)
        assert np.all(np.abs(y).max(1) <= bound)
        m_in = h.max(1)
        if L + 1 == 4:
            bound = np.maximum(bound, m_pe)
            m_in = np.maximum(m_in, m_pe)
        s = scale_of(bound)
    p = packed.astype(np.float64)
    off_sw = frag_offset(10) + 8 * 256
    off_sb = off_sw + 256
    off_db = off_sb + 4
    off_dwd = off_db + 128
    off_aw = off_dwd + 128 * 27
    off_ab = off_aw + 128 * 32
    off_rw = off_ab + 128
    off_rb = off_rw + 3 * 128
    sigma = np.maximum(h @ p[off_sw: off_sw + 256] + p[off_sb], 0)
    encd = O.positional_encoding(torch.from_numpy(d), 4).numpy().astype(np.float64)
    dvec = p[off_db: off_db + 128] + encd @ p[off_dwd: off_dwd + 128 * 27].reshape(128, 27).T
    appf = np.zeros(128) if app is None else p[off_ab: off_ab + 128] + app.astype(np.float64) @ \
        p[off_aw: off_aw + 128 * 32].reshape(128, 32).T
    hd = np.maximum(dense(8, inputs(8, h), s) + dvec, 0) + appf
    rgb = 1 / (1 + np.exp(-(hd @ p[off_rw: off_rw + 384].reshape(3, 128).T + p[off_rb: off_rb + 3])))
    return rgb, sigma[:, None]


def test_emulated_f16x3_kernel_matches_oracle(ref_state, app_vec):
    """The split arithmetic is fp32-accurate: the emulated f16x3 dataflow sits within the
    parity tolerance of the oracle and, per element, as close to a float64 evaluation as fp32."""
    packed = host_pack(ref_state)
    torch.manual_seed(5)
    x = torch.randn(256, 3) * 2
    d = torch.nn.functional.normalize(torch.randn(256, 3), dim=-1)
    st64 = {k: v.double() for k, v in ref_state.items()}
    for app in (None, app_vec):
        rgb, sigma = emulate_forward_f16x3(packed, x.numpy(), d.numpy(), None if app is None else app.numpy())
        rgb_o, sigma_o = O.nerf_forward(ref_state, x, d, app)
        np.testing.assert_allclose(rgb, rgb_o.numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(sigma, sigma_o.numpy(), rtol=1e-4, atol=1e-6)
        rgb64, _ = O.nerf_forward(st64, x.double(), d.double(), None if app is None else app.double())
        e16 = np.abs(rgb - rgb64.numpy()).max()
        e32 = np.abs(rgb_o.double().numpy() - rgb64.numpy()).max()
        assert e16 <= 4 * e32 + 1e-7, (e16, e32)


def host_pack_transposed(state):
    lib = _lib.load()
    ts = [state[k].contiguous().float() for k in O.STATE_KEYS]
    arr = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
    out = np.empty(lib.nerf_packed_transposed_floats(), dtype=np.float32)
    assert lib.nerf_pack_weights_transposed_host(arr, out.ctypes.data) == 0
    return out


def tfrag_matrix(packedT, mt):
    """Transposed fragment matrix mt as the backward kernel sees it: [i][slot], slot = 2*ks + h."""
    ks = 64 if mt == 7 else 128
    off = mt * 8 * 128 * 64
    blk = packedT[off: off + 8 * ks * 64].reshape(8, ks // 4, 2, 32, 4)
    return blk.transpose(0, 3, 1, 4, 2).reshape(256, ks * 2).astype(np.float64)


def test_transposed_fragments_are_permuted_weight_transposes(ref_state):
    packedT = host_pack_transposed(ref_state)
    assert packedT.size == 2 * (7 * 256 * 256 + 256 * 128) + 32
    for layer in range(1, 8):
        W = ref_state[f"pts_linears.{layer}.weight"].numpy()[:, :256]        # [out][in]
        cols = [act_feature(s // 2, s % 2) for s in range(256)]
        assert np.array_equal(tfrag_matrix(packedT, layer - 1), W.T[:, cols]), layer
    Wd = ref_state["dir_linear.weight"].numpy()[:, :256]                     # (128, 256)
    cols = [act_feature(s // 2, s % 2) for s in range(128)]
    assert np.array_equal(tfrag_matrix(packedT, 7), Wd.T[:, cols])


def test_transposed_split_f16_fragments(ref_state):
    """The split-f16 part of packedT (the data-gradient chain's weight stream): per matrix a
    power-of-two s_w with max |W s_w| < 2^14, hi = f16(W s_w) and lo = f16(W s_w - hi) in fragment
    order [group][k-step][tile][hi, lo][lane][8 halves], k index 32 (ks>>1) + 16 (ks&1) + 8 (j>>2) +
    4 h + (j&3); the matrices in consumption order (dir_linear's h-part, then trunk layers 7 .. 1);
    then the bound constants: each matrix's largest row L1 norm of W^T (x 1.0001) and max |w_sigma|."""
    packedT = host_pack_transposed(ref_state)
    base = 7 * 256 * 256 + 256 * 128
    consts = packedT[2 * base: 2 * base + 32]
    words = packedT[base: 2 * base].view(np.float16)
    off = 0
    for mt in (7, 6, 5, 4, 3, 2, 1, 0):
        if mt < 7:
            W = ref_state[f"pts_linears.{mt + 1}.weight"].numpy()[:, :256]       # [out][in]
        else:
            W = ref_state["dir_linear.weight"].numpy()[:, :256]
        WT = W.T.astype(np.float64)                                              # [in][out]
        sw, inv = float(consts[mt]), float(consts[8 + mt])
        assert sw * inv == 1.0 and np.log2(sw) == int(np.log2(sw))
        assert np.abs(WT).max() * sw < 2 ** 14 and np.abs(WT).max() * sw >= 2 ** 13
        KS = 16 if mt < 7 else 8
        n = 2 * KS * 4 * 2 * 64 * 8
        blk = words[off: off + n].astype(np.float64).reshape(2, KS, 4, 2, 2, 32, 8)   # g ks i part h c j
        off += n
        g, ks, i, h, c, j = np.meshgrid(np.arange(2), np.arange(KS), np.arange(4), np.arange(2), np.arange(32),
                                        np.arange(8), indexing="ij")
        row = 32 * (4 * g + i) + c
        col = 32 * (ks >> 1) + 16 * (ks & 1) + 8 * (j >> 2) + 4 * h + (j & 3)
        exp = WT[row, col] * sw
        hi, lo = blk[:, :, :, 0], blk[:, :, :, 1]
        assert np.array_equal(hi, exp.astype(np.float16).astype(np.float64)), mt
        assert np.abs(hi + lo - exp).max() <= 2.0 ** -10, mt      # |W s_w| < 2^14: split residual < 2^-11
        l1 = np.abs(WT).sum(1).max()
        assert l1 <= consts[16 + mt] <= l1 * 1.0002, mt              # rigorous bound: |W^T g| <= C max|g|
    assert consts[24] == np.abs(ref_state["density_head.weight"].numpy()).max()


def emulate_backward(packed, packedT, x, d, app, g_rgb, g_sigma):
    """The backward kernel's dataflow (csrc/train.hip mlp_backward_kernel) in float64: the
    transposed fragments applied to d pre-activations in accumulator order, returning the
    gradient with respect to the PE input and to every trunk pre-activation."""
    off_bias = frag_offset(10)
    off_sw = off_bias + 8 * 256
    off_sb = off_sw + 256
    off_db = off_sb + 4
    off_dwd = off_db + 128
    off_aw = off_dwd + 128 * 27
    off_ab = off_aw + 128 * 32
    off_rw = off_ab + 128
    off_rb = off_rw + 3 * 128
    p = packed.astype(np.float64)
    enc = O.positional_encoding(torch.from_numpy(x), 10).numpy().astype(np.float64)
    pe_slots = np.stack([enc[:, pe_feature(s // 2, s % 2)] if pe_feature(s // 2, s % 2) >= 0
                         else np.zeros(len(x)) for s in range(64)], 1)
    act = [act_feature(s // 2, s % 2) for s in range(256)]
    bias = p[off_bias: off_bias + 8 * 256].reshape(8, 256)
    hs = [np.maximum(pe_slots @ frag_matrix(packed, 0).T + bias[0], 0)]
    for m in range(1, 8):
        pre = hs[-1][:, act] @ frag_matrix(packed, m).T + bias[m]
        if m == 4:
            pre += pe_slots @ frag_matrix(packed, 9).T
        hs.append(np.maximum(pre, 0))
    h7 = hs[-1]
    sig = np.maximum(h7 @ p[off_sw: off_sw + 256] + p[off_sb], 0)
    encd = O.positional_encoding(torch.from_numpy(d), 4).numpy().astype(np.float64)
    dvec = p[off_db: off_db + 128] + encd @ p[off_dwd: off_dwd + 128 * 27].reshape(128, 27).T
    appf = np.zeros(128) if app is None else p[off_ab: off_ab + 128] + app.astype(np.float64) @ \
        p[off_aw: off_aw + 128 * 32].reshape(128, 32).T
    rdir = np.maximum(h7[:, act] @ frag_matrix(packed, 8).T + dvec, 0)
    hd = rdir + appf
    Wr = p[off_rw: off_rw + 384].reshape(3, 128)
    rgb = 1 / (1 + np.exp(-(hd @ Wr.T + p[off_rb: off_rb + 3])))
    # backward, mirroring the kernel
    dv = g_rgb * rgb * (1 - rgb)
    dhd = dv @ Wr
    dpre_dir = dhd * (rdir > 0)
    dh = dpre_dir[:, act[:128]] @ tfrag_matrix(packedT, 7).T
    dh += np.where(sig > 0, g_sigma, 0)[:, None] * p[off_sw: off_sw + 256]
    dpre = {}
    for layer in range(7, -1, -1):
        dpre[layer] = dh * (hs[layer] > 0)
        if layer:
            dh = dpre[layer][:, act] @ tfrag_matrix(packedT, layer - 1).T
    return dpre, dpre_dir, dhd


def test_emulated_backward_matches_autograd(ref_state, app_vec):
    """The transposed-fragment chain reproduces torch autograd on the oracle's forward."""
    packed, packedT = host_pack(ref_state), host_pack_transposed(ref_state)
    torch.manual_seed(6)
    x = torch.randn(128, 3, dtype=torch.float64) * 1.5
    d = torch.nn.functional.normalize(torch.randn(128, 3, dtype=torch.float64), dim=-1)
    g_rgb = torch.randn(128, 3, dtype=torch.float64)
    g_sigma = torch.randn(128, dtype=torch.float64)
    state = {k: v.double().requires_grad_(True) for k, v in ref_state.items()}
    pres = []
    rgb, sigma = O.nerf_forward(state, x, d, app_vec.double(), keep=pres)
    for t in pres:
        t.retain_grad()
    (rgb * g_rgb).sum().backward(retain_graph=True)
    (sigma[:, 0] * g_sigma).sum().backward()
    dpre, _, _ = emulate_backward(packed, packedT, x.numpy(), d.numpy(), app_vec.numpy(), g_rgb.numpy(),
                                  g_sigma.numpy())
    for layer in range(8):
        np.testing.assert_allclose(dpre[layer], pres[layer].grad.numpy(), rtol=1e-4, atol=1e-7)


def test_pe_sin_accuracy(tmp_path):
    """csrc/pe_sin.h (the f16x3 MLP's positional-encoding sin/cos) built for the host and compared
    with double-precision sin/cos at the arguments the encoding forms, 2^i x for |x| < 8, i < 10:
    within 1.6e-7 absolute (torch's float sin/cos sit within ~6e-8 of the same reference; the
    parity tolerance on the encoding is 2e-6)."""
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    src = tmp_path / "pe.cpp"
    src.write_text(r'''
#include "pe_sin.h"
#include <stdio.h>
#include <math.h>
int main() {
  unsigned s = 12345u;
  double worst = 0;
  for (int n = 0; n < 400000; ++n) {
    s = s * 1664525u + 1013904223u;
    const float x = ((s >> 8) / 16777216.0f) * 16.0f - 8.0f;
    for (int i = 0; i < 10; ++i)
      for (int h = 0; h < 2; ++h) {
        const float a = x * (float)(1 << i);
        const double ref = h ? cos((double)a) : sin((double)a);
        const double e = fabs((double)nerf::pe_sin_reduced(a, h) - ref);
        if (e > worst) worst = e;
      }
  }
  printf("%.6g\n", worst);
  return 0;
}
''')
    exe = tmp_path / "pe"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-I", os.path.join(REPO, "depth-aware-shader-effects-for-nerf_amd", "csrc"),
                    str(src), "-o", str(exe)], check=True)
    worst = float(subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout)
    assert worst < 1.6e-7, worst


@pytest.mark.skipif(os.environ.get("NERFMI_SANITIZED") == "1", reason="already the sanitized run")
def test_host_abi_under_asan_ubsan():
    """The host tests above, against the ASan + UBSan build of the C ABI (scripts/sanitize_host.sh:
    `make sanitize`: every -fsanitize on the host compilation, ~45 s from scratch on 8 cores, seconds
    when up to date): argument checks, workspace carving and the host packers run with every access and every
    undefined-behaviour check instrumented.  Part of the default CPU suite wherever hipcc exists."""
    import shutil
    import subprocess
    if not shutil.which("make") or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no hipcc to build the sanitized library")
    r = subprocess.run(["bash", os.path.join(REPO, "scripts", "sanitize_host.sh")], capture_output=True, text=True,
                       timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-3000:]


def test_render_chunk_plan():
    """nerf_render_rays / nerf_mlp_forward run a call of more than 2^30 samples per launch (the
    sample-parallel grids' limit) as ray chunks (capi.hip); the plan and the workspace are host
    arithmetic, checked here without a launch."""
    lib = _lib.load()
    assert lib.nerf_render_chunk_rays(64, 128) == (1 << 30) // 128
    assert lib.nerf_render_chunk_rays(64, 0) == (1 << 24)
    assert lib.nerf_render_chunk_rays(256, 1024) == (1 << 20)
    assert lib.nerf_render_chunk_rays(0, 0) == 0
    # the workspace covers one chunk: a 2^25-ray H1 call (2^32 fine samples) needs no more than
    # a 2^23-ray one, and an ordinary frame is unchanged
    big = lib.nerf_render_workspace_bytes(1 << 25, 64, 128)
    assert big == lib.nerf_render_workspace_bytes(1 << 23, 64, 128) > 0
    assert lib.nerf_render_workspace_bytes(640_000, 64, 128) < big
    # the appearance-row check runs before any chunk (app_rows must be 0, 1 or B)
    rc = lib.nerf_render_rays(None, None, None, 10, 2.0, 6.0, 64, 128, None, None, 1, None, None, 0, 0, None, 5,
                              None, None, None, None, None, None, None, 0, None)
    assert rc == 1 and b"app_rows" in lib.nerf_last_error()


def test_ray_longer_than_the_launch_limit_is_refused():
    """nerf_mlp_forward has no upper bound on N; when one ray's N samples exceed the per-launch sample
    limit the ray chunk would be 0 rays and the chunk loop would never advance.  It returns
    NERF_ERR_UNSUPPORTED instead (checked in a child process with the limit lowered to 4,096 by the
    NERFMI_MAX_LAUNCH_SAMPLES test hook, read once per process; no pointer is dereferenced)."""
    import subprocess
    import sys
    code = (
        "import sys, ctypes; sys.path.insert(0, %r)\n"
        "from nerfmi import _lib\n"
        "lib = _lib.load()\n"
        "assert lib.nerf_render_chunk_rays(5000, 0) == 0\n"
        "p = ctypes.c_void_p(16)\n"
        "rc = lib.nerf_mlp_forward(p, p, p, p, 3, 5000, p, p, p, None, 0, None)\n"
        "assert rc == 3 and b'launch limit' in lib.nerf_last_error(), (rc, lib.nerf_last_error())\n"
        "assert lib.nerf_mlp_forward(p, p, p, p, 0, 5000, p, p, p, None, 0, None) == 0\n"
        "print('ok')\n" % REPO)
    env = dict(os.environ, NERFMI_MAX_LAUNCH_SAMPLES="4096")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
