"""Kernel-level numerics through the C-ABI hooks, against plain PyTorch fp32
references of the same op (GEMM with every epilogue and tile config; attention
plain and causal at T = 50, 77, 577)."""
import numpy as np
import pytest
import torch

from clip_lora_match_amd import _capi as C

pytestmark = pytest.mark.gpu
DT = {"bfloat16": (torch.bfloat16, C.CLM_BF16), "float16": (torch.float16, C.CLM_F16)}


def _gemm(dtype, epi, cfg, A, W, out, bias=None, rs=None, cs=None):
    M, K = A.shape
    N = W.shape[0]
    p = lambda t: C.ptr(t) if t is not None else None  # noqa: E731
    C.check(C.lib().clm_gemm(A.device.index, DT[dtype][1], epi, cfg, C.ptr(A), A.stride(0), C.ptr(W), W.stride(0),
                             M, N, K, C.ptr(out), out.stride(0), p(bias), p(rs), p(cs),
                             C.stream_of(A.device)), "clm_gemm")


def _g4_ok(cfg, epi, N, K, ldo):
    """configs 13 / 14 (G4, k_gemm4.hip gemm4_supports): STORE / GELU with N, ldo multiples of 8,
    RESID with multiples of 4, whole 64-deep K-steps and at least two of them; anything else is
    refused (CLM_E_HIP)"""
    if cfg < 13:
        return True
    if K % 64 or K < 128 or N % 4 or ldo % 4:
        return False
    if epi == C.CLM_EPI_RESID:
        return True
    return epi in (C.CLM_EPI_STORE, C.CLM_EPI_GELU) and N % 8 == 0 and ldo % 8 == 0


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("cfg", list(range(15)) + [-1])
@pytest.mark.parametrize("shape", [(333, 200, 128), (1000, 768, 768), (77, 2304, 512), (97, 100, 64), (65, 50, 128),
                                   (300, 136, 800), (257, 64, 544)])
def test_gemm_epilogues_vs_torch(dtype, cfg, shape):
    """every tile config and epilogue vs torch; K = 800 / 544 (K % 64 == 32: the unmerged-LoRA
    32-wide K-extension, gemm_kernel configs only -- G2 configs must refuse it)"""
    M, N, K = shape
    td = DT[dtype][0]
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    kr = (K + 63) // 64 * 64   # rows readable to round_up(K, 64); the extra columns are never used
    A = torch.randn((M, kr), generator=g, device="cuda").to(td)[:, :K]
    W = (torch.randn((N, kr), generator=g, device="cuda") / K ** 0.5).to(td)[:, :K]
    bias = torch.randn(N, generator=g, device="cuda")
    ref = A.float() @ W.float().T + bias
    out = torch.empty((M, N), dtype=td, device="cuda")
    if K % 64 and 8 <= cfg <= 11:   # G2 runs whole 64-wide K-steps only
        with pytest.raises(Exception):
            _gemm(dtype, C.CLM_EPI_STORE, cfg, A, W, out, bias)
        return
    tol = 2e-2 if dtype == "bfloat16" else 4e-3

    def run(epi, o, *a):
        if not _g4_ok(cfg, epi, N, K, o.stride(0)):
            with pytest.raises(Exception):
                _gemm(dtype, epi, cfg, A, W, o, *a)
            return False
        _gemm(dtype, epi, cfg, A, W, o, *a)
        return True

    if run(C.CLM_EPI_STORE, out, bias):
        assert (out.float() - ref).abs().max() <= tol * ref.abs().max()
    refg = ref * torch.sigmoid(1.702 * ref)
    if run(C.CLM_EPI_GELU, out, bias):
        assert (out.float() - refg).abs().max() <= tol * refg.abs().max()
    h = torch.randn((M, N), generator=g, device="cuda")
    h0 = h.clone()
    if run(C.CLM_EPI_RESID, h, bias):
        assert (h - (h0 + ref)).abs().max() <= 1e-3 * ref.abs().max() + 1e-5
    rs = torch.rand(M, generator=g, device="cuda") + 0.5
    cs = torch.rand(N, generator=g, device="cuda") + 0.5
    sc = torch.empty((M, N), dtype=torch.float32, device="cuda")
    if run(C.CLM_EPI_SCORE, sc, None, rs, cs):
        refs = (A.float() @ W.float().T) * rs[:, None] * cs[None, :]
        assert (sc - refs).abs().max() <= 1e-4 * refs.abs().max() + 1e-6


@pytest.mark.parametrize("epi", ["STORE", "GELU", "RESID", "SCORE"])
@pytest.mark.parametrize("N", [192, 200])
def test_gemm_row_invariance_and_bounds(epi, N):
    """Every tile config gives bit-identical rows (same K order), a row's value does not
    depend on M or on which rows share its tile (sub-batches == full batch), and nothing
    outside [M, N) of the output is written (padding columns of ldo > N, rows >= M)."""
    dtype, M, K, ldo, split = "float16", 119, 256, N + 24, 51
    code = getattr(C, f"CLM_EPI_{epi}")
    g = torch.Generator(device="cuda").manual_seed(N)
    A = torch.randn((M, K), generator=g, device="cuda").half()
    W = (torch.randn((N, K), generator=g, device="cuda") / K ** 0.5).half()
    bias = torch.randn(N, generator=g, device="cuda") if epi != "SCORE" else None
    rs = torch.rand(M, generator=g, device="cuda") + 0.5 if epi == "SCORE" else None
    cs = torch.rand(N, generator=g, device="cuda") + 0.5 if epi == "SCORE" else None
    odt = torch.float32 if epi in ("RESID", "SCORE") else torch.float16
    init = torch.randn((M + 40, ldo), generator=g, device="cuda").to(odt)
    ref = None
    for cfg in list(range(C.lib().clm_gemm_num_configs())) + [-1]:
        if not _g4_ok(cfg, code, N, K, ldo):
            continue
        out = init.clone()
        _gemm(dtype, code, cfg, A, W, out[:M], bias, rs, cs)
        assert torch.equal(out[:, N:], init[:, N:]) and torch.equal(out[M:], init[M:]), f"cfg {cfg} wrote outside"
        parts = init.clone()   # two sub-batches of rows [0, split) and [split, M)
        _gemm(dtype, code, cfg, A[:split], W, parts[:split], bias, rs[:split] if rs is not None else None, cs)
        _gemm(dtype, code, cfg, A[split:], W, parts[split:M], bias, rs[split:] if rs is not None else None, cs)
        assert torch.equal(parts, out), f"cfg {cfg}: sub-batch rows differ from the full batch"
        if ref is None:
            ref = out
        assert torch.equal(out, ref), f"cfg {cfg} differs from cfg 0"


@pytest.mark.parametrize("shape", [(8200, 2100, 64), (8200, 2100, 192), (8200, 2098, 128), (8200, 2112, 320)])
def test_gemm_persistent_multi_tile(shape):
    """Grids with more tiles than resident workgroups: each workgroup walks several tiles with
    one LDS-DMA ring across tile boundaries (K = 64: every K-step ends a tile; N = 2098: the
    ragged scalar epilogue). Must equal the one-tile-per-workgroup grid bit for bit (debug
    flag 4) and the fp32 reference."""
    M, N, K = shape
    g = torch.Generator(device="cuda").manual_seed(K)
    A = torch.randn((M, K), generator=g, device="cuda").half()
    W = (torch.randn((N, K), generator=g, device="cuda") / K ** 0.5).half()
    bias = torch.randn(N, generator=g, device="cuda")
    ref = A.float() @ W.float().T + bias
    h0 = torch.randn((M, N), generator=g, device="cuda")
    try:
        for cfg in list(range(C.lib().clm_gemm_num_configs())) + [-1]:
            for epi in (C.CLM_EPI_STORE, C.CLM_EPI_RESID):
                if not _g4_ok(cfg, epi, N, K, N):
                    continue
                outs = []
                for dbg in (0, 4):
                    C.lib().clm_debug_set(dbg)
                    out = h0.clone() if epi == C.CLM_EPI_RESID else torch.empty((M, N), dtype=torch.half, device="cuda")
                    _gemm("float16", epi, cfg, A, W, out, bias)
                    outs.append(out)
                assert torch.equal(outs[0], outs[1]), f"cfg {cfg} epi {epi}: persistent grid differs"
                want = h0 + ref if epi == C.CLM_EPI_RESID else ref
                assert (outs[0].float() - want).abs().max() <= 4e-3 * ref.abs().max(), f"cfg {cfg} epi {epi}"
    finally:
        C.lib().clm_debug_set(0)


def test_gemm_asymmetric_identity():
    """A = I catches a transposed C write (cdna_hip_programming §3 'A=I-check with ASYMMETRIC B')."""
    n = 128
    A = torch.eye(n, device="cuda", dtype=torch.float16)
    W = torch.arange(n * n, device="cuda", dtype=torch.float32).reshape(n, n).remainder(97).half()
    out = torch.empty((n, n), dtype=torch.float16, device="cuda")
    for cfg in range(C.lib().clm_gemm_num_configs()):
        _gemm("float16", C.CLM_EPI_STORE, cfg, A, W, out)
        assert torch.equal(out, W.T.contiguous())


def _attn_ref(qkv, B, T, H, causal):
    d = H * 64
    x = qkv.float().view(B, T, 3, H, 64)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    s = q @ k.transpose(-1, -2)      # q already carries the 64^-1/2 scale
    if causal:
        s = s + torch.triu(torch.full((T, T), float("-inf"), device=s.device), 1)
    return (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B * T, d)


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("B,T,H,causal,ramp", [(3, 50, 12, False, 0), (2, 77, 8, True, 0), (2, 77, 8, False, 0),
                                               (1, 577, 16, False, 0), (2, 130, 2, True, 0), (1, 1, 2, True, 0),
                                               (2, 130, 2, False, 0), (2, 160, 3, False, 0), (1, 193, 2, False, 0),
                                               (2, 250, 4, False, 0), (1, 577, 2, False, 1), (1, 577, 2, False, -1),
                                               (1, 700, 3, False, 1), (1, 577, 2, False, 2), (2, 300, 2, False, 2)])
def test_attention_vs_torch(dtype, B, T, H, causal, ramp):
    """T > 128 non-causal runs the 32x32x16 online-softmax kernel: tail tiles of 2 / 32 / 1 / 58
    keys, and key magnitudes ramped up (the running max grows tile after tile: every rescale
    fires), steeply up (ramp 2: the scores outgrow the lazy shift by far more than 2^15, so the
    exact-rescale path runs on later tiles too) or down (none after the first tile)."""
    td = DT[dtype][0]
    g = torch.Generator(device="cuda").manual_seed(T * H)
    qkv = torch.randn((B * T, 3 * H * 64), generator=g, device="cuda")
    qkv[:, : H * 64] *= 0.125 * 3
    if ramp:
        t = torch.linspace(0.0, 1.0, T, device="cuda").repeat(B)
        f = 0.5 + (2.0 if abs(ramp) == 1 else 12.0) * (t if ramp > 0 else 1.0 - t)
        qkv[:, H * 64: 2 * H * 64] *= f[:, None]
    qkv = qkv.to(td)
    out = torch.full((B * T, H * 64 + 64), 7.0, device="cuda").to(td)
    C.check(C.lib().clm_attention(0, DT[dtype][1], int(causal), C.ptr(qkv), C.ptr(out), out.stride(0), B, T, H,
                                  C.stream_of(qkv.device)), "clm_attention")
    ref = _attn_ref(qkv, B, T, H, causal)
    err = (out[:, : H * 64].float() - ref).abs().max().item()
    assert err < (3e-2 if dtype == "bfloat16" else 4e-3), err
    assert (out[:, H * 64:].float() == 7.0).all()   # columns past d untouched


@pytest.mark.parametrize("B,T,H,ramp", [(1, 577, 16, 0), (2, 130, 2, 0), (1, 193, 2, 1), (2, 300, 2, 2),
                                         (1, 577, 2, -1), (1, 700, 3, 2)])
def test_attention_q_log2e_vs_torch(B, T, H, ramp):
    """CLM_ATTN_Q_LOG2E (the engine's form for the L/14 image tower): q carries log2(e) too, the
    running shift enters the score MFMA chain as a bf16 operand. Inputs as in the unfolded test,
    q scaled by log2 e in fp32 and rounded once to bf16; the fp32 reference takes that same
    rounded q with log2 e divided back out (so both see one q), same bar; the first-step and
    2^15-sum rescale paths are exercised by the ramps."""
    g = torch.Generator(device="cuda").manual_seed(T * H + 1)
    qkv = torch.randn((B * T, 3 * H * 64), generator=g, device="cuda")
    qkv[:, : H * 64] *= 0.125 * 3
    if ramp:
        t = torch.linspace(0.0, 1.0, T, device="cuda").repeat(B)
        f = 0.5 + (2.0 if abs(ramp) == 1 else 12.0) * (t if ramp > 0 else 1.0 - t)
        qkv[:, H * 64: 2 * H * 64] *= f[:, None]
    folded = qkv.clone()
    folded[:, : H * 64] *= 1.4426950408889634
    folded = folded.to(torch.bfloat16)
    ref_in = folded.float()   # the reference sees the same rounded q (log2 e divided back out in fp32)
    ref_in[:, : H * 64] /= 1.4426950408889634
    out = torch.full((B * T, H * 64 + 64), 7.0, device="cuda").to(torch.bfloat16)
    C.check(C.lib().clm_attention_ex(0, C.CLM_BF16, C.CLM_ATTN_Q_LOG2E, C.ptr(folded), C.ptr(out), out.stride(0), B,
                                     T, H, C.stream_of(qkv.device)), "clm_attention_ex")
    ref = _attn_ref(ref_in, B, T, H, False)
    err = (out[:, : H * 64].float() - ref).abs().max().item()
    assert err < 3e-2, err
    assert (out[:, H * 64:].float() == 7.0).all()


@pytest.mark.parametrize("folded", [True, False])
def test_attention_very_negative_first_tile(folded):
    """every query's logits against the first 32 keys are ~-190 (log2 domain ~-275, below the
    -128 where exp2(-shift) overflows): the first step's rescale must not turn the zero O and sum
    into NaN (the log2e-folded form started its shift at 0)"""
    B, T, H = 1, 577, 2
    g = torch.Generator(device="cuda").manual_seed(11)
    qkv = torch.randn((B * T, 3 * H * 64), generator=g, device="cuda") * 0.3
    qkv[:, : H * 64] = 1.0                      # q: every dim 1
    qkv[:32, H * 64: 2 * H * 64] = -3.0         # first 32 keys: q . k = -192 for every query
    q_in = qkv.clone()
    if folded:
        q_in[:, : H * 64] *= 1.4426950408889634
    q_in = q_in.to(torch.bfloat16)
    ref_in = q_in.float()
    if folded:
        ref_in[:, : H * 64] /= 1.4426950408889634
    out = torch.zeros((B * T, H * 64), device="cuda", dtype=torch.bfloat16)
    C.check(C.lib().clm_attention_ex(0, C.CLM_BF16, C.CLM_ATTN_Q_LOG2E if folded else 0, C.ptr(q_in), C.ptr(out),
                                     out.stride(0), B, T, H, C.stream_of(qkv.device)), "clm_attention_ex")
    assert torch.isfinite(out.float()).all()
    err = (out.float() - _attn_ref(ref_in, B, T, H, False)).abs().max().item()
    assert err < 3e-2, err


def test_attention_causal_switch_keeps_meaning():
    """clm_attention's `causal` is a 0 / non-0 switch: 5 means causal, like 1"""
    B, T, H = 2, 77, 2
    g = torch.Generator(device="cuda").manual_seed(5)
    qkv = torch.randn((B * T, 3 * H * 64), generator=g, device="cuda").to(torch.float16)
    o1 = torch.zeros((B * T, H * 64), device="cuda", dtype=torch.float16)
    o5 = torch.ones_like(o1)
    for c, o in ((1, o1), (5, o5)):
        C.check(C.lib().clm_attention(0, C.CLM_F16, c, C.ptr(qkv), C.ptr(o), o.stride(0), B, T, H,
                                      C.stream_of(qkv.device)), "clm_attention")
    assert torch.equal(o1, o5)


@pytest.mark.parametrize("dtype,flags,T", [("float16", 2, 577), ("bfloat16", 3, 577), ("bfloat16", 2, 128),
                                           ("bfloat16", 4, 577)])
def test_attention_q_log2e_refused(dtype, flags, T):
    """the log2(e) form exists only for the bf16, non-causal, T > 128 kernel; unknown flags refused"""
    qkv = torch.zeros((T, 3 * 64), dtype=DT[dtype][0], device="cuda")
    out = torch.zeros((T, 64), dtype=DT[dtype][0], device="cuda")
    rc = C.lib().clm_attention_ex(0, DT[dtype][1], flags, C.ptr(qkv), C.ptr(out), 64, 1, T, 1, C.stream_of(qkv.device))
    assert rc == C.CLM_E_ARG


def _rounding_probe(n, seed):
    """fp32 values that stress the fp32 -> 16-bit RNE conversion: every binade from fp16
    subnormals to past the fp16 overflow threshold, exact half-way ties, zero (acc + bias turns a -0 bias into +0, so none here)."""
    g = np.random.default_rng(seed)
    mag = np.exp2(g.uniform(-30, 18, n)).astype(np.float32)
    v = (mag * g.choice([-1.0, 1.0], n)).astype(np.float32)
    ties = (np.float32(1.0) + np.float32(2.0 ** -11) * (2 * g.integers(0, 1024, 64) + 1)).astype(np.float32)
    v[:64] = ties                                   # half-way between two fp16 values
    v[64:128] = (ties - 1.0) * np.float32(2.0 ** -14)   # ties in the fp16 subnormal range
    v[128:136] = [0.0, -1e-30, 65504.0, 65519.0, 65520.0, -65520.0, 6e-8, -3e-8]
    return torch.from_numpy(v)


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("N", [1024, 1023])
def test_epilogue_rounding_matches_torch(dtype, N):
    """A bias-only GEMM (A = W = 0) stores fp32 bias values through the 16-bit epilogue: the
    packed 16-B path (N % 8 == 0) and the scalar tail path (N odd) round exactly as torch's
    .to(dtype), in every tile configuration (batch invariance rests on this)."""
    td = DT[dtype][0]
    M, K = 80, 64
    bias = _rounding_probe(N, N).cuda()
    A = torch.zeros((M, K), dtype=td, device="cuda")
    W = torch.zeros((N, K), dtype=td, device="cuda")
    want = bias.to(td).view(torch.int16).expand(M, N)
    for cfg in list(range(C.lib().clm_gemm_num_configs())) + [-1]:
        if not _g4_ok(cfg, C.CLM_EPI_STORE, N, K, N):
            continue
        out = torch.empty((M, N), dtype=td, device="cuda")
        _gemm(dtype, C.CLM_EPI_STORE, cfg, A, W, out, bias=bias)
        got = out.view(torch.int16)
        bad = (got != want).nonzero()
        assert bad.numel() == 0, (cfg, [(float(bias[j]), int(got[i, j]), int(want[i, j])) for i, j in bad[:4].tolist()])


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("epi", ["STORE", "GELU", "RESID"])
def test_gemm_configs_bit_identical(dtype, epi):
    """Every tile configuration computes each output row with the same K order and the same
    epilogue arithmetic, so all give bit-identical results: the encoder's batch invariance
    (a row's embedding does not depend on which batch, or which M tile, it lands in)."""
    td = DT[dtype][0]
    M, N, K = 300, 768, 768
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randn((M, K), generator=g, device="cuda").to(td)
    W = (torch.randn((N, K), generator=g, device="cuda") / K ** 0.5).to(td)
    bias = torch.randn(N, generator=g, device="cuda")
    h0 = torch.randn((M, N), generator=g, device="cuda")
    e = getattr(C, f"CLM_EPI_{epi}")
    first = None
    for cfg in range(C.lib().clm_gemm_num_configs()):
        out = h0.clone() if epi == "RESID" else torch.empty((M, N), dtype=td, device="cuda")
        _gemm(dtype, e, cfg, A, W, out, bias=bias)
        if first is None:
            first = out
        else:
            d = (out.float() - first.float()).abs()
            assert torch.equal(out, first), (cfg, float(d.max()), d.amax(1).nonzero().flatten()[:8].tolist())


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("epi,N,K", [("STORE", 2304, 768), ("RESID", 768, 768), ("GELU", 3072, 768),
                                     ("RESID", 768, 3072), ("STORE", 1536, 512), ("GELU", 2048, 512),
                                     ("RESID", 512, 2048)])
def test_gemm_rows_independent_of_batch(dtype, epi, N, K):
    """The encoder's GEMM shapes at the heuristic config, run on row sets of different sizes
    (a tower's M = batch x tokens, and the pruned last layer's M = batch): a row's output bits do
    not depend on M or on where the row sits in its M tile."""
    td = DT[dtype][0]
    g = torch.Generator(device="cuda").manual_seed(N + K)
    Mfull = 250
    A = torch.randn((Mfull, K), generator=g, device="cuda").to(td)
    W = (torch.randn((N, K), generator=g, device="cuda") / K ** 0.5).to(td)
    bias = torch.randn(N, generator=g, device="cuda")
    h0 = torch.randn((Mfull, N), generator=g, device="cuda")
    e = getattr(C, f"CLM_EPI_{epi}")

    def run(rows):
        out = h0[rows].clone() if epi == "RESID" else torch.empty((len(rows), N), dtype=td, device="cuda")
        _gemm(dtype, e, -1, A[rows].contiguous(), W, out, bias=bias)
        return out

    ref = run(list(range(Mfull)))
    for rows in (list(range(200, 250)), list(range(150, 250)), [249, 3, 77, 200, 5], [249], list(range(50, 250))):
        got = run(rows)
        d = (got.float() - ref[rows].float()).abs()
        assert torch.equal(got, ref[rows]), (len(rows), float(d.max()), d.amax(1).nonzero().flatten()[:8].tolist())


def _ln(dtype, x, g, b, eps=1e-5):
    M, d = x.shape
    y = torch.empty((M, d), dtype=DT[dtype][0], device="cuda")
    C.check(C.lib().clm_layernorm(0, DT[dtype][1], C.ptr(x), x.stride(0), M, d, C.ptr(g), C.ptr(b), eps, C.ptr(y),
                                  y.stride(0), C.stream_of(x.device)), "clm_layernorm")
    return y


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("d", [512, 768, 1024])
def test_layernorm_vs_torch_and_row_invariant(dtype, d):
    """The encoder LayerNorm kernel vs torch fp32 LayerNorm (one 16-bit rounding of the output
    apart), and every row's bits independent of the row count and of the row's position (pairs of
    rows share a wave)."""
    g = torch.Generator(device="cuda").manual_seed(d)
    M = 301
    x = torch.randn((M, d), generator=g, device="cuda") * 3 + torch.randn((M, 1), generator=g, device="cuda") * 5
    gam = torch.randn(d, generator=g, device="cuda")
    bet = torch.randn(d, generator=g, device="cuda")
    y = _ln(dtype, x, gam, bet)
    ref = torch.nn.functional.layer_norm(x, (d,), gam, bet, 1e-5)
    ulp = 2.0 ** (-8 if dtype == "bfloat16" else -11)
    assert ((y.float() - ref).abs() <= ulp * ref.abs() + 1e-6).all()
    for rows in ([300], [1, 0], list(range(1, 301)), [5, 6, 7], list(range(300, -1, -1))):
        assert torch.equal(_ln(dtype, x[rows].contiguous(), gam, bet), y[rows]), rows


def test_c_abi_under_host_sanitizers_with_device():
    """The prebuilt host-sanitizer harness (csrc/Makefile `sanitize`, ASan + UBSan on the host
    half) over the index lifecycle and the host-buffer entry points, results checked against
    scalar host references inside the harness."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "clip-lora-match_amd", "host_check")
    assert os.path.exists(exe), "build it with make -C clip-lora-match_amd/csrc sanitize"
    p = subprocess.run([exe], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "argument + device checks, 0 failure(s)" in p.stdout
