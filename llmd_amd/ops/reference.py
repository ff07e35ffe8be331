"""Plain PyTorch fp32 reference implementations of every llmd_amd HIP op.

Used (a) as the numerics oracle in the kernel tests and (b) as the execution
path for CPU tensors (CPU CI, the GPU-free simulator). They follow exactly the
semantics documented in the corresponding ``csrc/ops/*.hip`` file, including
the paged KV layout ``[num_blocks, Hkv, block_size, D]`` per layer.
"""
from __future__ import annotations

import math

import torch


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * inv * w.float()).to(x.dtype)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    """In place: residual += x (rounded to x.dtype); x = rmsnorm(residual) * w."""
    r = (x.float() + residual.float()).to(residual.dtype)
    residual.copy_(r)
    x.copy_(rms_norm(r, w, eps))


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def fused_add_layer_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float):
    """In place: residual += x (rounded to x.dtype); x = layernorm(residual) * w + b."""
    r = (x.float() + residual.float()).to(residual.dtype)
    residual.copy_(r)
    x.copy_(layer_norm(r, w, b, eps))


FP8_MAX = 448.0


def to_cache(x: torch.Tensor, cache_dtype, scale: float = 1.0) -> torch.Tensor:
    """Cache storage conversion: bf16 as is; fp8 e4m3fn = saturate(x / scale)."""
    if cache_dtype == torch.float8_e4m3fn:
        return (x.float() / scale).clamp(-FP8_MAX, FP8_MAX).to(cache_dtype)
    return x.to(cache_dtype)


def rope_cache(qkv, positions, cos_sin, Hq, Hkv, D, slots, k_cache, v_cache, neox=True, k_scale=1.0,
               v_scale=1.0):
    """Rotate Q (in place in qkv) and K, write K/V into the paged cache at slots."""
    T = qkv.shape[0]
    if T == 0:
        return
    rot = cos_sin.shape[1]
    half = rot // 2
    cs = cos_sin[positions].float()  # [T, rot]
    cos, sin = cs[:, :half], cs[:, half:]
    heads = qkv[:, : (Hq + 2 * Hkv) * D].view(T, Hq + 2 * Hkv, D)
    qk = heads[:, : Hq + Hkv, :rot].float()
    if neox:
        a, b = qk[..., :half], qk[..., half:]
    else:
        a, b = qk[..., 0::2], qk[..., 1::2]
    c, s = cos[:, None, :], sin[:, None, :]
    oa, ob = a * c - b * s, b * c + a * s
    if neox:
        out = torch.cat([oa, ob], -1)
    else:
        out = torch.stack([oa, ob], -1).flatten(-2)
    out = out.to(qkv.dtype)
    heads[:, :Hq, :rot] = out[:, :Hq]
    k_full = heads[:, Hq : Hq + Hkv].clone()
    k_full[..., :rot] = out[:, Hq:]
    v_full = heads[:, Hq + Hkv : Hq + 2 * Hkv]
    bs = k_cache.shape[2]
    valid = slots >= 0
    if valid.any():
        sl = slots[valid]
        blk, off = sl // bs, sl % bs
        k_cache[blk, :, off, :] = to_cache(k_full[valid], k_cache.dtype, k_scale)
        v_cache[blk, :, off, :] = to_cache(v_full[valid], v_cache.dtype, v_scale)


def gated_act(x: torch.Tensor, mode: int = 0, alpha: float = 1.702, limit: float = 7.0):
    xf = x.float()
    if mode == 2:
        g, u = xf[:, 0::2], xf[:, 1::2]
        g = g.clamp(max=limit)
        u = u.clamp(-limit, limit)
        return ((u + 1) * g * torch.sigmoid(alpha * g)).to(x.dtype)
    F = x.shape[1] // 2
    g, u = xf[:, :F], xf[:, F:]
    if mode == 0:
        a = torch.nn.functional.silu(g)
    else:
        a = torch.nn.functional.gelu(g, approximate="tanh")
    return (a * u).to(x.dtype)


def _gather_kv(k_cache, v_cache, block_table, L, k_scale=1.0, v_scale=1.0):
    bs = k_cache.shape[2]
    nb = (L + bs - 1) // bs
    blocks = block_table[:nb].long()
    k = k_cache[blocks].permute(1, 0, 2, 3).reshape(k_cache.shape[1], nb * bs, -1)[:, :L]
    v = v_cache[blocks].permute(1, 0, 2, 3).reshape(v_cache.shape[1], nb * bs, -1)[:, :L]
    return k.float() * k_scale, v.float() * v_scale  # [Hkv, L, D]


def attention_ref(q, k, v, q_pos, scale, window=0, sinks=None):
    """q [Tq, Hq, D], k/v [Hkv, L, D] (positions 0..L-1); causal by q_pos."""
    Hq, Hkv = q.shape[1], k.shape[0]
    G = Hq // Hkv
    kk = k.repeat_interleave(G, 0)  # [Hq, L, D]
    vv = v.repeat_interleave(G, 0)
    s = torch.einsum("thd,hld->htl", q.float(), kk) * scale
    L = k.shape[1]
    kpos = torch.arange(L, device=q.device)
    mask = kpos[None, :] <= q_pos[:, None]
    if window and window > 0:
        mask &= kpos[None, :] > (q_pos[:, None] - window)
    s = s.masked_fill(~mask[None], float("-inf"))
    if sinks is not None:
        sk = sinks.float()[:, None, None].expand(Hq, s.shape[1], 1)
        s = torch.cat([s, sk], -1)
        p = torch.softmax(s, -1)[..., :-1]
    else:
        p = torch.softmax(s, -1)
    return torch.einsum("htl,hld->thd", p, vv)


def paged_decode(q, k_cache, v_cache, block_tables, seq_lens, Hq, Hkv, D, scale, window=0,
                 sinks=None, k_scale=1.0, v_scale=1.0):
    B = q.shape[0]
    out = torch.empty(B, Hq, D, dtype=q.dtype, device=q.device)
    for b in range(B):
        L = int(seq_lens[b])
        k, v = _gather_kv(k_cache, v_cache, block_tables[b], L, k_scale, v_scale)
        qb = q[b, : Hq * D].view(1, Hq, D)
        o = attention_ref(qb, k, v, torch.tensor([L - 1], device=q.device), scale, window, sinks)
        out[b] = o[0].to(q.dtype)
    return out.view(B, Hq * D)


def paged_prefill(q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, Hq, Hkv, D, scale,
                  window=0, sinks=None, k_scale=1.0, v_scale=1.0):
    T = q.shape[0]
    out = torch.zeros(T, Hq * D, dtype=q.dtype, device=q.device)
    for i in range(len(q_len)):
        qs, ql, ctx = int(q_start[i]), int(q_len[i]), int(ctx_len[i])
        if ql == 0:
            continue
        k, v = _gather_kv(k_cache, v_cache, block_tables[i], ctx, k_scale, v_scale)
        qi = q[qs : qs + ql, : Hq * D].view(ql, Hq, D)
        qpos = torch.arange(ctx - ql, ctx, device=q.device)
        o = attention_ref(qi, k, v, qpos, scale, window, sinks)
        out[qs : qs + ql] = o.reshape(ql, Hq * D).to(q.dtype)
    return out


def sample(logits, temps=None, generator=None):
    """Greedy for temp<=0 else multinomial from softmax(logits/T). Returns (ids, logprob)."""
    lf = logits.float()
    logp = torch.log_softmax(lf, -1)
    ids = lf.argmax(-1)
    if temps is not None:
        t = temps.float()
        sm = t > 0
        if sm.any():
            probs = torch.softmax(lf[sm] / t[sm, None], -1)
            ids = ids.clone()
            ids[sm] = torch.multinomial(probs, 1, generator=generator).squeeze(-1)
    return ids, logp.gather(-1, ids[:, None]).squeeze(-1)


def topk_topp_mask(logits, topk=None, topp=None, temps=None):
    lf = logits
    B, V = lf.shape
    for b in range(B):
        row = lf[b]
        t = float(temps[b]) if temps is not None and float(temps[b]) > 0 else 1.0
        k = int(topk[b]) if topk is not None else 0
        p = float(topp[b]) if topp is not None else 1.0
        keep = torch.ones(V, dtype=torch.bool, device=lf.device)
        if 0 < k < V:
            thr = torch.topk(row, k).values[-1]
            keep &= row >= thr
        if p < 1.0:
            probs = torch.softmax(row / t, -1)
            sp, idx = torch.sort(probs, descending=True)
            cum = torch.cumsum(sp, 0)
            n = int((cum < p).sum().item()) + 1
            thr = row[idx[min(n, V) - 1]]
            keep &= row >= thr
        row.masked_fill_(~keep, float("-inf"))
    return lf


def rope_cos_sin(rot_dim: int, max_pos: int, base: float = 10000.0, scaling: dict | None = None,
                 device="cpu") -> torch.Tensor:
    """[max_pos, rot_dim] f32 table: cos in [:, :rot/2], sin in [:, rot/2:].

    Supports Llama-3 frequency scaling ("llama3") and linear scaling; YaRN for
    DeepSeek / gpt-oss is handled by ``yarn_inv_freq``.
    """
    inv_freq = 1.0 / (base ** (torch.arange(0, rot_dim, 2, dtype=torch.float64) / rot_dim))
    mscale = 1.0
    if scaling:
        kind = scaling.get("rope_type", scaling.get("type"))
        if kind == "llama3":
            factor = scaling["factor"]
            lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
            old = scaling.get("original_max_position_embeddings", 8192)
            lo_wl, hi_wl = old / lo, old / hi
            wl = 2 * math.pi / inv_freq
            smooth = (old / wl - lo) / (hi - lo)
            scaled = torch.where(wl > lo_wl, inv_freq / factor, inv_freq)
            mid = (1 - smooth) * inv_freq / factor + smooth * inv_freq
            is_mid = (wl <= lo_wl) & (wl >= hi_wl)
            inv_freq = torch.where(is_mid, mid, scaled)
        elif kind == "linear":
            inv_freq = inv_freq / scaling["factor"]
        elif kind == "yarn":
            inv_freq, mscale = yarn_inv_freq(rot_dim, base, scaling)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv_freq)
    return torch.cat([f.cos() * mscale, f.sin() * mscale], -1).float().to(device)


def yarn_inv_freq(rot_dim, base, sc):
    factor = sc["factor"]
    old = sc.get("original_max_position_embeddings", 4096)
    beta_fast, beta_slow = sc.get("beta_fast", 32), sc.get("beta_slow", 1)

    def corr_dim(nrot):
        return (rot_dim * math.log(old / (nrot * 2 * math.pi))) / (2 * math.log(base))

    low = max(math.floor(corr_dim(beta_fast)), 0)
    high = min(math.ceil(corr_dim(beta_slow)), rot_dim - 1)
    pos_freqs = base ** (torch.arange(0, rot_dim, 2, dtype=torch.float64) / rot_dim)
    extra, inter = 1.0 / pos_freqs, 1.0 / (factor * pos_freqs)
    ramp = torch.clamp((torch.arange(rot_dim // 2, dtype=torch.float64) - low) / max(high - low, 1e-3), 0, 1)
    mask = 1 - ramp
    inv = inter * (1 - mask) + extra * mask
    def get_mscale(ms):
        return 0.1 * ms * math.log(factor) + 1.0 if factor > 1 else 1.0

    if sc.get("mscale_all_dim"):  # DeepSeek: cos/sin scaled by mscale/mscale_all_dim
        m = get_mscale(sc.get("mscale", 1.0)) / get_mscale(sc["mscale_all_dim"])
    else:
        m = get_mscale(sc.get("mscale", 1.0))
    return inv, m


def yarn_softmax_mscale(sc: dict | None) -> float:
    """DeepSeek YaRN: the softmax scale is multiplied by mscale_all_dim-mscale squared."""
    if not sc or sc.get("rope_type", sc.get("type")) != "yarn" or not sc.get("mscale_all_dim"):
        return 1.0
    f = sc["factor"]
    m = 0.1 * sc["mscale_all_dim"] * math.log(f) + 1.0 if f > 1 else 1.0
    return m * m


def mla_rope_cache(q, q_lat, kv_c, k_pe, positions, cos_sin, H, slots, cache, kv_scale=1.0):
    """q [T, H*192] (nope 128 | pe 64) -> q_lat[:, h*576+512:+64] = rope(q_pe);
    cache.view(-1, 576)[slot] = [kv_c | rope(k_pe)] (GPT-J interleaved pairs)."""
    T = q.shape[0]
    cs = cos_sin[positions.long()].float()
    cos, sin = cs[:, :32], cs[:, 32:]

    def rot(x):  # x [..., 64] pairs (2i, 2i+1)
        x0, x1 = x[..., 0::2].float(), x[..., 1::2].float()
        c, s_ = cos.view(T, *([1] * (x.dim() - 2)), 32), sin.view(T, *([1] * (x.dim() - 2)), 32)
        y = torch.stack([x0 * c - x1 * s_, x0 * s_ + x1 * c], -1)
        return y.flatten(-2)

    qp = q[:, : H * 192].view(T, H, 192)[:, :, 128:]
    q_lat.view(T, H, 576)[:, :, 512:] = rot(qp).to(q_lat.dtype)
    bs = cache.shape[1]
    ok = slots >= 0
    row = to_cache(torch.cat([kv_c.float(), rot(k_pe)], -1), cache.dtype, kv_scale)
    sl = slots[ok].long()
    cache[sl // bs, sl % bs] = row[ok]


# ---------------------------------------------------------------- MoE references
def moe_topk(logits, k, scoring=0, bias=None, n_group=1, topk_group=1, renorm=False, routed_scale=1.0):
    """scoring: 0 softmax, 1 sigmoid, 2 softmax over the selected top-k logits (gpt-oss)."""
    lf = logits.float()
    if scoring == 0:
        sc = torch.softmax(lf, -1)
    elif scoring == 1:
        sc = torch.sigmoid(lf)
    else:
        sc = lf
    sel = sc + (bias.float() if bias is not None else 0.0)
    if scoring == 2:
        sel = lf + (bias.float() if bias is not None else 0.0)
    T, E = lf.shape
    if n_group > 1:
        g = sel.view(T, n_group, E // n_group)
        gs = g.topk(min(2, E // n_group), -1).values.sum(-1)
        keep = torch.zeros(T, n_group, dtype=torch.bool, device=lf.device)
        keep.scatter_(1, gs.topk(topk_group, -1).indices, True)
        sel = sel.masked_fill(~keep.repeat_interleave(E // n_group, 1), float("-inf"))
    ids = sel.topk(k, -1).indices
    w = sc.gather(-1, ids)
    if scoring == 2:
        w = torch.softmax(lf.gather(-1, ids), -1)
    elif renorm:
        w = w / w.sum(-1, keepdim=True)
    return ids.int(), (w * routed_scale).float()


def moe_forward(x, ids, wts, w1, w2, act=0, alpha=1.702, limit=7.0, b1=None, b2=None):
    """Dense reference: w1 [E, 2F, d] with interleaved gate/up rows, w2 [E, d, F]."""
    T, d = x.shape
    out = torch.zeros(T, d, dtype=torch.float32, device=x.device)
    xf = x.float()
    for t in range(T):
        for j in range(ids.shape[1]):
            e = int(ids[t, j])
            if e < 0:
                continue
            h = w1[e].float() @ xf[t]
            if b1 is not None:
                h = h + b1[e].float()
            g, u = h[0::2], h[1::2]
            if act == 2:
                g = g.clamp(max=limit)
                u = u.clamp(-limit, limit)
                a = (u + 1) * g * torch.sigmoid(alpha * g)
            else:
                a = torch.nn.functional.silu(g) * u
            a = a.to(x.dtype).float()
            y = w2[e].float() @ a
            if b2 is not None:
                y = y + b2[e].float()
            y = y.to(x.dtype).float()
            out[t] += float(wts[t, j]) * y
    return out.to(x.dtype)


def mla_attention(q, cache, block_tables, row_seq, row_len, H, scale, kv_scale=1.0):
    """Absorbed MLA: q [R, H*576], cache [blocks, bs, 576] -> out [R, H*512]
    (value = first 512 dims of the cached latent)."""
    R = q.shape[0]
    bs = cache.shape[1]
    out = torch.zeros(R, H, 512, dtype=torch.float32, device=q.device)
    qf = q[:, : H * 576].float().view(R, H, 576)
    for r in range(R):
        L = int(row_len[r])
        bt = block_tables[int(row_seq[r])]
        idx = torch.arange(L, device=q.device)
        kv = cache[bt[idx // bs].long(), idx % bs].float() * kv_scale  # [L, 576]
        s = (qf[r] @ kv.T) * scale                           # [H, L]
        p = torch.softmax(s, -1)
        out[r] = p @ kv[:, :512]
    return out.view(R, H * 512).to(q.dtype)


def lora_bgmv(y, x, A, B, slot):
    """y[t] += B[slot[t]] @ (A[slot[t]] @ x[t]) (slot 0 = no adapter); in place."""
    s = slot[: x.shape[0]].long()
    on = s > 0
    if bool(on.any()):
        xa = torch.einsum("ti,tri->tr", x[on].float(), A[s[on]].float())
        d = torch.einsum("tr,tor->to", xa, B[s[on]].float())
        y[on] = (y[on].float() + d).to(y.dtype)
    return y
