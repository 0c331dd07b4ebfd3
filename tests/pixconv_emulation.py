"""CPU emulation of the pixel-major GridNet kernels (microbeast_amd/ops/pixconv.py): the same
bf16 maths as pixconv.hip with per-pixel torch loops -- the oracle the CPU tests and the GPU
numerics tests compare the kernels against (test code, not a product path). tests/conftest.py
registers it with ``pixconv.set_emulation``; each function receives the calling op's
arguments and locals as keywords."""
import torch

from microbeast_amd.ops import pixconv as pc  # (its _BF / _view at call time: tests patch _BF)


def pconv(*, A, a_ps, a_bs, cin, B, tab, N, M, C, c_ps, c_bs, bias, relu, a_relu, mask, cells, gather, **_):
    if cells is not None or gather is not None:
        return _pconv_sparse_ref(A, a_ps, a_bs, cin, B, tab, N, M, C, c_ps, c_bs, bias, relu,
                                 a_relu, mask, cells, gather)
    tabc = tab.t.cpu()
    for z in range(tabc.shape[0]):
        P, cnt = int(tabc[z, 0]), int(tabc[z, 1])
        acc = torch.zeros(M, N, dtype=torch.float32)
        for j in range(cnt):
            e = int(tabc[z, 2 + j])
            q, t = e >> 8, e & 255
            a = pc._view(A, a_ps, a_bs, M, cin, q).float()
            if a_relu:
                a = a.clamp_min(0)
            b = B.reshape(-1)[t * N * cin:(t + 1) * N * cin].view(N, cin).float()
            acc += a @ b.t()
        if bias is not None:
            acc += bias.float()
        if relu:
            acc = acc.clamp_min(0)
        out = acc.to(C.dtype)
        if mask is not None:
            m = pc._view(mask, c_ps, c_bs, M, N, P).float() > 0
            out = torch.where(m, out, torch.zeros_like(out))
        pc._view(C, c_ps, c_bs, M, N, P).copy_(out)
    return C


def rows_colsum(*, self, Z, ld, C, out, **_):
    nact = int(self.totals[0])
    out.view(-1).copy_(Z.view(-1, ld)[:nact, :C].float().sum(0))
    return


def pwgrad(*, g, g_ps, g_bs, O, x, x_ps, x_bs, I, tab, M, gmap, out, x_relu, cells, ntap, **_):
    tabc = tab.t.cpu()
    dw = torch.zeros(ntap, O, I, dtype=torch.float32)
    for t in range(ntap):
        for j in range(int(tabc[t, 0])):
            e = int(tabc[t, 1 + j])
            P, q = e >> 16, e & 0xFFFF
            if cells is not None:
                o, nr = int(cells.bucket_off[P]), int(cells.bucket_cnt[P])
                gv = torch.as_strided(g.reshape(-1), (nr, O), (g_bs, 1), o * g_bs).float()
                xv = pc._view(x, x_ps, x_bs, M, I, q)[cells.rowimg[o:o + nr].long()].float()
            else:
                gv = pc._view(g, g_ps, g_bs, M, O, P).float()
                xv = pc._view(x, x_ps, x_bs, M, I, q).float()
            if x_relu:
                xv = xv.clamp_min(0)
            dw[t] += gv.t() @ xv
    m = gmap.long()
    out.view(-1).copy_(torch.where(m >= 0, dw.reshape(-1)[m.clamp(min=0)], 0.0))
    return out


def pwgrad_all(*, g, g_ps, g_bs, O, x, x_ps, x_bs, I, ftab, ntap, M, gmap, out, x_relu, bias_out, **_):
    tabc = ftab.t.cpu()
    dw = torch.zeros(ntap, O, I, dtype=torch.float32)
    if bias_out is not None:
        bias_out.zero_()
    for z in range(tabc.shape[0]):
        P = int(tabc[z, 0])
        gv = pc._view(g, g_ps, g_bs, M, O, P).float()
        for j in range(int(tabc[z, 1])):
            e = int(tabc[z, 2 + j])
            q, t = e >> 8, e & 255
            xv = pc._view(x, x_ps, x_bs, M, I, q).float()
            if x_relu:
                xv = xv.clamp_min(0)
            dw[t] += gv.t() @ xv
        if bias_out is not None:
            bias_out += gv.float().sum(0)
    m = gmap.long()
    out.view(-1).copy_(torch.where(m >= 0, dw.reshape(-1)[m.clamp(min=0)], 0.0))
    return out


def ppool_fwd(*, y, H, W, n, C, out, idx, Ho, Wo, **_):
    yv = y.view(H, W, n, C).float()
    best = torch.full((Ho, Wo, n, C), float("-inf"))
    bi = torch.zeros(Ho, Wo, n, C, dtype=torch.uint8)
    for ky in range(3):
        for kx in range(3):
            for Y in range(Ho):
                yy = 2 * Y - 1 + ky
                if not 0 <= yy < H:
                    continue
                for X in range(Wo):
                    xx = 2 * X - 1 + kx
                    if not 0 <= xx < W:
                        continue
                    v = yv[yy, xx]
                    upd = v > best[Y, X]
                    best[Y, X] = torch.where(upd, v, best[Y, X])
                    bi[Y, X] = torch.where(upd, ky * 3 + kx, bi[Y, X].int()).to(torch.uint8)
    out.copy_(best.view(Ho * Wo, n, C))
    idx.copy_(bi.view(Ho * Wo, n, C))
    return out, idx


def ppool_bwd(*, g1, n1, g2, n2, pooled, idx, H, W, n, C, Ho, Wo, **_):
    g = torch.zeros(Ho * Wo, n, C)
    g[:, :n1] += g1.float().view(Ho * Wo, n1, C)
    if g2 is not None:
        g[:, :n2] += g2.float().view(Ho * Wo, n2, C)
    g = g * (pooled.float() > 0)
    dy = torch.zeros(H, W, n, C)
    gv, iv = g.view(Ho, Wo, n, C), idx.view(Ho, Wo, n, C)
    for Y in range(Ho):
        for X in range(Wo):
            for ky in range(3):
                for kx in range(3):
                    yy, xx = 2 * Y - 1 + ky, 2 * X - 1 + kx
                    if 0 <= yy < H and 0 <= xx < W:
                        dy[yy, xx] += gv[Y, X] * (iv[Y, X] == ky * 3 + kx)
    return dy.view(H * W, n, C).to(pc._BF)


def colsum(*, x, C, out, c0, out1, **_):
    s = x[:, :C].float().sum(0)
    out.view(-1).copy_(s[:c0])
    if out1 is not None:
        out1.view(-1).copy_(s[c0:])
    return


def map_gather(*, segs, **_):
    for src, dst, m in segs:
        v = src.reshape(-1)[m.long().clamp(min=0)] * (m >= 0)
        dst.view(-1).copy_(v.reshape(-1))
    return


def gemm_nt(*, a, b, bias, out_dtype, **_):
    y = a.float() @ b.float().t()
    if bias is not None:
        y = y + bias
    return y.to(out_dtype)


def value_bwd(*, dv, h, w2, gw2, gb2, gadd, R, K, **_):
    dvf = dv.float().reshape(R, 1)
    gw2.view(-1).copy_((dvf * h.float()).sum(0))
    gb2.view(-1).copy_(dvf.sum())
    d = dvf * w2.reshape(1, K)
    if gadd is not None:
        d[:gadd.shape[0]] += gadd.float()
    return (d * (h > 0)).to(pc._BF)


def _pconv_sparse_ref(A, a_ps, a_bs, cin, B, tab, N, M, C, c_ps, c_bs, bias, relu, a_relu, mask,
                      cells, gather):
    tabc = tab.t.cpu()
    for z in range(tabc.shape[0]):
        P, cnt = int(tabc[z, 0]), int(tabc[z, 1])
        if cells is not None:
            o, nr = int(cells.bucket_off[z]), int(cells.bucket_cnt[z])
            imgs = cells.rowimg[o:o + nr].long()
        else:
            nr = M
        acc = torch.zeros(nr, N, dtype=torch.float32)
        for j in range(cnt):
            e = int(tabc[z, 2 + j])
            q, t = e >> 8, e & 255
            if cells is not None:
                a = pc._view(A, a_ps, a_bs, M, cin, q)[imgs].float()
            else:
                rows = gather.cellrow[q * M:(q + 1) * M].long()
                src = torch.as_strided(A.reshape(-1), (gather.cap, cin), (a_bs, 1), 0)
                a = torch.where((rows >= 0)[:, None], src[rows.clamp(min=0)].float(), 0.0)
            if a_relu:
                a = a.clamp_min(0)
            b = B.reshape(-1)[t * N * cin:(t + 1) * N * cin].view(N, cin).float()
            acc += a @ b.t()
        if bias is not None:
            acc += bias.float()
        if relu:
            acc = acc.clamp_min(0)
        out = acc.to(C.dtype)
        if cells is not None:
            torch.as_strided(C.reshape(-1), (nr, N), (c_bs, 1), o * c_bs).copy_(out)
        else:
            if mask is not None:
                m = pc._view(mask, c_ps, c_bs, M, N, P).float() > 0
                out = torch.where(m, out, torch.zeros_like(out))
            pc._view(C, c_ps, c_bs, M, N, P).copy_(out)
    return C
