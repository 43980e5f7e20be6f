"""Model of K5a's LDS insert (round 5): 16 waves x 64 lanes x 8 keys into a 16 Ki-slot
linear-probing table; counts the compare-and-swap wave instructions of the probe-round insert
(lds_insert: per key position, rounds while any lane collides) against a streamed insert
(each lane one CAS per step).  The streamed form was built on this model's 27 -> 15 and
measured SLOWER: the model counts instructions, not round trips or VALU."""
# Simulate K5a's LDS insert: 16 waves x 64 lanes x 8 keys (8 Ki keys) into a 16 Ki-slot linear-probing table.
# Count wave CAS instructions: current (per position: 1 + max extra probes over lanes) vs streamed (max over lanes of attempts).
import numpy as np
rng = np.random.default_rng(1)
N = 100_000_000
# zipf(0.99) ranks via inverse cdf on a truncated support (sampling approximation)
M = 10_000_000
w = np.arange(1, M + 1, dtype=np.float64) ** -0.99
cdf = np.cumsum(w); cdf /= cdf[-1]
perm = rng.permutation(M).astype(np.uint32) * 7 + 3
def fmix32(x):
    x = np.uint64(x)
    x ^= x >> np.uint64(16); x = (x * np.uint64(0x85ebca6b)) & np.uint64(0xffffffff)
    x ^= x >> np.uint64(13); x = (x * np.uint64(0xc2b2ae35)) & np.uint64(0xffffffff)
    x ^= x >> np.uint64(16)
    return int(x)
def run(SLOTS, KPT=8, waves=16, trials=20, dist="zipf", twochoice=False):
    cur_tot = str_tot = 0; distinct = 0
    for t in range(trials):
        n = waves * 64 * KPT
        if dist == "zipf":
            keys = perm[np.searchsorted(cdf, rng.random(n))]
        else:
            keys = rng.integers(0, N, n).astype(np.uint32)
        distinct += len(np.unique(keys))
        keys = keys.reshape(waves, KPT, 64)  # wave, position, lane
        table = {}
        # model: waves interleave position by position (round-robin), each instruction atomically in lane order
        # attempts per (wave, pos, lane)
        att = np.zeros((waves, KPT, 64), dtype=np.int32)
        for q in range(KPT):
            for wv in range(waves):
                for l in range(64):
                    k = int(keys[wv, q, l]); h = fmix32(k) & (SLOTS - 1); a = 1
                    while True:
                        o = table.get(h)
                        if o is None:
                            table[h] = k; break
                        if o == k: break
                        h = (h + 1) & (SLOTS - 1); a += 1
                    att[wv, q, l] = a
        cur = att.max(axis=2).sum(axis=1)          # per wave: sum over positions of max attempts
        stream = att.sum(axis=1).max(axis=1)        # per wave: max over lanes of total attempts
        cur_tot += cur.mean(); str_tot += stream.mean()
    return distinct / trials, cur_tot / trials, str_tot / trials
for slots in (16384, 32768):
    for dist in ("zipf", "uniform"):
        d, c, s = run(slots, dist=dist, trials=4)
        print(f"SLOTS {slots} {dist}: distinct {d:.0f}  CAS instr/wave current {c:.1f}  streamed {s:.1f}")
