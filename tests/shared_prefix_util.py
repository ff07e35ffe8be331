"""Block tables whose sequences share cached prefixes (test helper)."""
import numpy as np


def shared_tables(prefix_groups, suffixes, bs, seed=0):
    """prefix_groups: list of (prefix tokens, member count); suffixes: per member
    extra tokens (cycled). Returns (block table rows [B, W] int32, lens [B], pool
    blocks). Members of a group map their first prefix//bs blocks onto the same
    physical blocks; the rest of every row is private. Pool order is shuffled."""
    rng = np.random.default_rng(seed)
    rows, lens = [], []
    nxt = 0
    si = 0
    for P, n in prefix_groups:
        pre = list(range(nxt, nxt + P // bs))
        nxt += P // bs
        for _ in range(n):
            S = suffixes[si % len(suffixes)]
            si += 1
            L = P + S
            own = -(-L // bs) - len(pre)
            rows.append(pre + list(range(nxt, nxt + own)))
            nxt += own
            lens.append(L)
    W = max(len(r) for r in rows)
    perm = rng.permutation(nxt)
    bt = np.zeros((len(rows), W), np.int32)
    for i, r in enumerate(rows):
        bt[i, :len(r)] = perm[r]
    return bt, np.asarray(lens, np.int32), nxt
