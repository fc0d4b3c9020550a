# numpy emulation of the 4-lanes-per-column median (csrc/common_mode.hip, CQ = 4): the exact lane /
# DPP algorithm checked against np.median on random columns (ties, empty, tiny, odd sizes).
import numpy as np
INF = np.float32(np.inf)

def bitonic_sort_64(z):
    z = list(z)
    j = 32
    while j >= 1:
        for i in range(64):
            if (i & j) == 0:
                a, b = z[i], z[i + j]
                z[i], z[i + j] = min(a, b), max(a, b)
        j //= 2
    return z

def quad_median(col, part):
    """col: R values; part: bool participants. Emulates the 4-lane algorithm; returns (lo, hi, cnt)."""
    R = len(col)
    M4 = (R + 3) // 4
    N = 4 * M4
    lanes = []
    for q in range(4):
        x = []
        for i in range(M4):
            r = q * M4 + i
            x.append(np.float32(col[r]) if (r < R and part[r]) else np.nan)
        lanes.append(x)
    inv = [sum(1 for v in x if np.isnan(v)) for x in lanes]
    total_inv = sum(inv)
    cnt = N - total_inv
    a = total_inv >> 1
    for q in range(4):
        prefix = sum(inv[:q])
        neg_budget = min(inv[q], max(0, a - prefix))
        ninv = 0
        for i in range(M4):
            if np.isnan(lanes[q][i]):
                lanes[q][i] = -INF if ninv < neg_budget else INF
                ninv += 1
        lanes[q] = sorted(lanes[q])
    # level 1: merge-split with q^1, negate lower, pad +inf to 64, bitonic merge, unmap
    xs = [None] * 4
    for q in range(4):
        own, par = lanes[q], lanes[q ^ 1]
        lower = (q & 1) == 0
        y = [min(own[i], par[M4 - 1 - i]) if lower else max(own[i], par[M4 - 1 - i]) for i in range(M4)]
        z = [-v if lower else v for v in y] + [INF] * (64 - M4)
        z = bitonic_sort_64(z)
        xs[q] = [(-z[M4 - 1 - i]) if lower else z[i] for i in range(M4)]
    # level 2: lanes 0,1 compute parts with partner lanes 3,2 (quad_perm [3,2,1,0])
    e = xs[2][M4 - 1]
    p88, p87 = [], []
    for q in (0, 1):
        own, P = xs[q], xs[3 - q]
        k88 = min(max(own[t], P[M4 - 1 - t]) for t in range(M4))
        k87 = min([max(own[t], P[M4 - 2 - t]) for t in range(M4 - 1)] + [INF])
        extra = min(P[M4 - 1], max(own[M4 - 1], e)) if q == 0 else own[M4 - 1]
        p88.append(k88)
        p87.append(min(k87, extra))
    kth88, kth87 = min(p88), min(p87)
    lo = kth87
    hi = kth87 if (cnt & 1) else kth88
    return lo, hi, cnt

def run(trials=3000, seed=0):
  rng = np.random.default_rng(seed)
  bad = 0
  for trial in range(trials):
      R = int(rng.choice([176, 175, 173, 16, 9, 4, 1, 8, 12]))
      col = rng.normal(0, 10, R).astype(np.float32)
      if trial % 7 == 0:
          col = np.round(col)            # ties
      part = rng.random(R) < rng.choice([0.0, 0.05, 0.5, 0.9, 1.0])
      lo, hi, cnt = quad_median(col, part)
      assert cnt == part.sum()
      if cnt == 0:
          continue
      med = np.float32((np.float32(lo) + np.float32(hi)) * np.float32(0.5))
      ref = np.float32(np.median(col[part]))
      if med != ref:
          bad += 1
          if bad < 5:
              print("MISMATCH", R, cnt, med, ref)
  return bad


if __name__ == "__main__":
    print("mismatches:", run())
