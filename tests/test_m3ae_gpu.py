"""GPU parity of the frozen M3AE text encoder (csrc/m3ae.hip) through the C ABI: each building
block against a float64 torch evaluation of the same op, and the whole encoder against the
oracle's op-for-op torch-fp32 restatement of forward_representation over the FULL padded
sequence (oracle/m3ae_text.py; parity unpinned by reference fixtures -- none exist).
Tolerance 1e-4 (BASELINE north_star) relative to max(1, |ref|)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-4


def _close(got, ref, tol=TOL):
    got, ref = got.detach().double().cpu(), ref.detach().double().cpu()
    err = (got - ref).abs().max().item()
    assert err <= tol * max(1.0, ref.abs().max().item()), err


def _encoder(vocab, depth, d=384, heads=6, seed=0):
    from mmre.m3ae import M3AETextEncoder
    torch.manual_seed(seed)
    enc = M3AETextEncoder(vocab, d, depth, heads)
    with torch.no_grad():
        for n, p in enc.named_parameters():
            if "layer_norm" in n:
                p.add_(0.1 * torch.randn_like(p))
            elif n.endswith("bias"):
                p.copy_(0.02 * torch.randn_like(p))
    return enc


def _rows(lens, L, vocab, seed, holes=False):
    g = torch.Generator().manual_seed(seed)
    tok = torch.randint(0, vocab, (len(lens), L), generator=g).to(torch.int32)
    msk = torch.ones(len(lens), L)
    for b, n in enumerate(lens):
        msk[b, :n] = 0
    if holes:  # interior padding as well (the mask is used as given, submodule.py:174-177)
        msk[-1, 2:5] = 1
    return tok, msk


@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("m,k,n", [(1, 384, 384), (100, 384, 1152), (77, 1536, 384), (130, 1280, 1280)])
def test_linear_matches_float64(epi, m, k, n):
    from mmre._lib import call, ptr, stream_ptr
    g = torch.Generator().manual_seed(m + k + n)
    a = torch.randn(m, k, generator=g)
    w = torch.randn(n, k, generator=g) / k ** 0.5
    b = 0.1 * torch.randn(n, generator=g)
    r = torch.randn(m, n, generator=g)
    ref = a.double() @ w.double().T + b.double()
    if epi == 1:
        ref = torch.nn.functional.gelu(ref)
    if epi == 2:
        ref = r.double() + ref
    ad, wd, bd = a.to(DEV), w.to(DEV), b.to(DEV)
    out = r.to(DEV).clone() if epi == 2 else torch.empty(m, n, device=DEV)
    call("mmre_m3ae_linear", epi, ptr(ad), m, k, ptr(wd), n, ptr(bd), ptr(out) if epi == 2 else None, ptr(out),
         stream_ptr(DEV))
    torch.cuda.synchronize()
    _close(out, ref)


@pytest.mark.parametrize("d", [384, 768, 1024, 1280])
def test_layernorm_matches_float64(d):
    from mmre._lib import call, ptr, stream_ptr
    g = torch.Generator().manual_seed(d)
    x = 3.0 * torch.randn(37, d, generator=g) + 0.5
    w, b = 1 + 0.1 * torch.randn(d, generator=g), 0.1 * torch.randn(d, generator=g)
    ref = torch.nn.functional.layer_norm(x.double(), (d,), w.double(), b.double(), eps=1e-5)
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    y = torch.empty_like(xd)
    call("mmre_m3ae_layernorm", ptr(xd), 37, d, ptr(wd), ptr(bd), 1e-5, ptr(y), stream_ptr(DEV))
    torch.cuda.synchronize()
    _close(y, ref, 1e-5)


@pytest.mark.parametrize("heads,hd", [(6, 64), (16, 80)])
def test_attention_matches_float64(heads, hd):
    """Packed rows of sequences of 1 .. 321 rows (chunk edges 64 / 65, the 16-row query blocks),
    softmax((q k^T) * hd^-0.5) v per sequence and head; and the CLS-only form of the last block."""
    from mmre._lib import call, ptr, stream_ptr
    lens = [1, 5, 16, 17, 64, 65, 200, 321]
    D = heads * hd
    off = np.r_[0, np.cumsum(lens)].astype(np.int32)
    g = torch.Generator().manual_seed(hd)
    qkv = torch.randn(int(off[-1]), 3 * D, generator=g)
    scale = hd ** -0.5
    ref = torch.empty(int(off[-1]), D, dtype=torch.float64)
    for s, n in enumerate(lens):
        blk = qkv[off[s]:off[s + 1]].double().view(n, 3, heads, hd).permute(1, 2, 0, 3)
        q, k, v = blk[0], blk[1], blk[2]
        p = torch.softmax((q @ k.transpose(-2, -1)) * scale, -1)
        ref[off[s]:off[s + 1]] = (p @ v).permute(1, 0, 2).reshape(n, D)
    qd, od = qkv.to(DEV), torch.from_numpy(off).to(DEV)
    out = torch.full((int(off[-1]), D), float("nan"), device=DEV)
    call("mmre_m3ae_attention", ptr(qd), ptr(od), len(lens), max(lens), heads, hd, float(np.float32(scale)), 0,
         ptr(out), stream_ptr(DEV))
    cls = torch.empty(len(lens), D, device=DEV)
    call("mmre_m3ae_attention", ptr(qd), ptr(od), len(lens), max(lens), heads, hd, float(np.float32(scale)), 1,
         ptr(cls), stream_ptr(DEV))
    torch.cuda.synchronize()
    _close(out, ref, 1e-5)
    _close(cls, ref[torch.from_numpy(off[:-1]).long()], 1e-5)


@pytest.mark.parametrize("L,lens,holes", [(64, [0, 1, 7, 33, 64], True), (320, [12, 320, 3], False)])
def test_encoder_matches_oracle(L, lens, holes):
    """CLS of the padding-free / CLS-only HIP encoder vs the oracle over the full padded rows,
    with empty, full and interior-padded rows; the dedupe of adjacent repeats is exact."""
    import m3ae_text as om
    vocab = 500
    enc = _encoder(vocab, depth=2)
    tok, msk = _rows(lens, L, vocab, seed=L, holes=holes)
    ref, _ = om.forward_representation_text(enc.state_dict(), tok, msk, 6)
    enc = enc.to(DEV)
    tok_d, msk_d = tok.to(DEV), msk.to(DEV)
    cls = enc.encode(tok_d, msk_d)
    torch.cuda.synchronize()
    _close(cls, ref[:, 0])
    # adjacent repeats (different ids on padded positions) are encoded once; rows are
    # independent of their packing: everything bit-identical
    tok2 = torch.where(msk_d > 0, torch.randint_like(tok_d, 0, vocab), tok_d)
    rep = enc.encode(torch.stack([tok_d, tok2, tok_d], 1).flatten(0, 1), msk_d.repeat_interleave(3, 0))
    far = enc.encode(torch.cat([tok_d, tok2, tok_d]), torch.cat([msk_d, msk_d, msk_d]))
    nodup = enc.encode(tok_d, msk_d, dedupe=False)
    torch.cuda.synchronize()
    n = len(lens)
    assert torch.equal(rep, cls.repeat_interleave(3, 0)) and torch.equal(far, cls.repeat(3, 1))
    assert torch.equal(nodup, cls)


def test_encoder_small_full_depth():
    """M3AE-small (d 384, 12 blocks, 6 heads; utils.py:127-134) on 320-token rows."""
    import m3ae_text as om
    vocab = 1000
    enc = _encoder(vocab, depth=12)
    tok, msk = _rows([9, 40, 1], 320, vocab, seed=5)
    ref, _ = om.forward_representation_text(enc.state_dict(), tok, msk, 6)
    enc = enc.to(DEV)
    cls, _ = enc.forward_representation(None, tok.to(DEV), msk.to(DEV))
    torch.cuda.synchronize()
    assert cls.shape == (3, 1, 384)
    _close(cls[:, 0], ref[:, 0])


def test_encoder_rejects_bad_ids():
    from mmre._lib import MMREError
    enc = _encoder(50, depth=1).to(DEV)
    tok = torch.tensor([[1, 2, 60, 3]], dtype=torch.int32, device=DEV)
    msk = torch.zeros(1, 4, device=DEV)
    with pytest.raises(MMREError):
        enc.encode(tok, msk)
    msk[0, 2] = 1  # the out-of-range id sits on a padded position: ignored, like the reference
    assert torch.isfinite(enc.encode(tok, msk)).all()


def test_plan_dedupes_adjacent_repeats_and_counts_bad_ids():
    """mmre_m3ae_plan: a row equal to the previous one on its padding pattern and unpadded tokens
    (ids on padded positions may differ) shares its unique sequence; packed offsets count the
    CLS row + unpadded tokens; unpadded ids outside [0, vocab) are counted."""
    from mmre._lib import call, lib, ptr, stream_ptr
    L = 8
    rows = [([1, 2, 3, 0, 0, 0, 0, 0], 3), ([1, 2, 3, 9, 9, 9, 9, 9], 3), ([1, 2, 3, 0, 0, 0, 0, 0], 4),
            ([1, 2, 3, 0, 0, 0, 0, 0], 4), ([5, 5, 5, 5, 5, 5, 5, 5], 8), ([1, 2, 3, 0, 0, 0, 0, 0], 3)]
    tok = torch.tensor([r for r, _ in rows], dtype=torch.int32, device=DEV)
    msk = torch.tensor([[0.0] * n + [1.0] * (L - n) for _, n in rows], device=DEV)
    B = len(rows)
    plan = torch.full((int(lib().mmre_m3ae_plan_size(B)),), -7, dtype=torch.int32, device=DEV)
    call("mmre_m3ae_plan", ptr(tok), ptr(msk), B, L, 1, 10, ptr(plan), stream_ptr(DEV))
    p = plan.cpu().numpy()
    assert list(p[:B]) == [0, 0, 1, 1, 2, 3]                  # uniq
    assert list(p[B:B + 4]) == [0, 2, 4, 5]                   # src rows of the unique sequences
    assert list(p[2 * B:2 * B + 5]) == [0, 4, 9, 18, 22]      # packed offsets
    assert list(p[3 * B + 1:3 * B + 5]) == [4, 22, 9, 0]      # n_unique, n_rows, max_rows, bad ids
    call("mmre_m3ae_plan", ptr(tok), ptr(msk), B, L, 0, 5, ptr(plan), stream_ptr(DEV))  # no dedupe, vocab 5
    p = plan.cpu().numpy()
    assert list(p[:B]) == list(range(B))
    assert list(p[3 * B + 1:3 * B + 5]) == [6, 4 + 4 + 5 + 5 + 9 + 4, 9, 8]  # the eight 5s are out of range
