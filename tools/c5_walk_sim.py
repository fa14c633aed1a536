"""Step counts of k_part_acc's walk (csrc/part.hip) against a kind-uniform walk (VERDICT r05
item 6), simulated over real block digit structure (tools/part_entries.py's scalars: r-point
weights, y-point a c / b c mod l, block sums; signed radix-2^16 digits split into 8-bit windows).

Each of a block's 64 lanes walks one unit of windows 0..15 and one of 16..31, paired as
k_part_sort pairs them (r-th largest low unit with r-th smallest high unit).  A unit is its
buckets in ascending order: E (run += entry) per entry, B (acc += run) per bucket boundary.

  lockstep (the product): one branch-free 9 M step per action, steps = max over lanes.
  uniform: a lane at a boundary parks a snapshot of run in a FIFO of K slots (no arithmetic)
           and goes on with entries; entry steps cost 7 M (run += affine Niels point), boundary
           steps 9 M (acc += a parked snapshot, every lane with one); a boundary step runs when
           at least `thresh` lanes are blocked (FIFO full or unit ended with snapshots left) or
           no lane has an entry.  Parking stores, FIFO bookkeeping and the LDS the FIFO needs
           (K x 160 B per lane) are NOT charged: the ratio is the best case.

Usage: python3 tools/c5_walk_sim.py [blocks] > profiles/rNN_c5_walk_sim.json
"""
import json
import random, sys
sys.path.insert(0, '/root/repo/tools')
from part_entries import recode16, split8, L

def block_digits(rng, proofs=128):
    """per 8-bit window (32 windows): list of |byte digits| (nonzero) of the block's entries"""
    win = [[] for _ in range(32)]
    sa = sb = 0
    def add16(digs):
        for w, d in enumerate(digs):
            lo, hi = split8(d)
            if lo: win[2*w].append(abs(lo))
            if hi: win[2*w+1].append(abs(hi))
    for _ in range(proofs):
        words = [rng.getrandbits(16) for _ in range(16)]
        signed = [w - 65536 if w >= 32768 else w for w in words]
        a = sum(signed[k] << (16*k) for k in range(8)) % L
        b = sum(signed[8+k] << (16*k) for k in range(8)) % L
        c, s = rng.randrange(L), rng.randrange(1, L)
        add16(signed[:8]); add16(signed[8:])
        add16(recode16(a*c % L)); add16(recode16(b*c % L))
        sa, sb = (sa + a*s) % L, (sb + b*s) % L
    add16(recode16(sa)); add16(recode16(sb))
    return win

def units(win):
    """64 low units (windows 0..15 x 4 shares of 32 buckets), 64 high (16..31); top window 16 buckets, 4 per share"""
    lo, hi = [], []
    for v in range(32):
        width = 4 if v == 31 else 32
        cnt = [0]*129
        for d in win[v]: cnt[d] += 1
        for h in range(4):
            seq = []
            for k in range(width*h, width*h+width):
                # bucket k holds digit k+1? buckets 1..128 -> index k = d-1
                seq += ['E']*cnt[k+1] + ['B']
            (lo if v < 16 else hi).append(seq)
    return lo, hi

def lanes(lo, hi):
    lo = sorted(lo, key=len, reverse=True); hi = sorted(hi, key=len)
    return [lo[r] + ['U'] + hi[r] + ['U'] for r in range(64)]   # U: end of unit (drain)

def lockstep(L_):
    return max(sum(1 for x in s if x != 'U') for s in L_)

def uniform(L_, K, thresh):
    n = len(L_)
    pos = [0]*n; fifo = [0]*n
    e_steps = b_steps = 0
    while True:
        # free parking: lanes at B with FIFO space park (advance), repeatedly
        for i in range(n):
            s = L_[i]
            while pos[i] < len(s) and s[pos[i]] == 'B' and fifo[i] < K:
                fifo[i] += 1; pos[i] += 1
            if pos[i] < len(s) and s[pos[i]] == 'U' and fifo[i] == 0:
                pos[i] += 1
                while pos[i] < len(s) and s[pos[i]] == 'B' and fifo[i] < K:
                    fifo[i] += 1; pos[i] += 1
        can_e = [pos[i] < len(L_[i]) and L_[i][pos[i]] == 'E' for i in range(n)]
        blocked = sum(1 for i in range(n) if fifo[i] > 0 and not can_e[i])
        done = all(pos[i] >= len(L_[i]) and fifo[i] == 0 for i in range(n))
        if done: break
        if not any(can_e) or blocked >= thresh:
            b_steps += 1
            for i in range(n):
                if fifo[i]: fifo[i] -= 1
        else:
            e_steps += 1
            for i in range(n):
                if can_e[i]: pos[i] += 1
    return e_steps, b_steps

def main(blocks=8, seed=7):
    import statistics
    rng = random.Random(seed)
    res = []
    for _ in range(blocks):
        lo, hi = units(block_digits(rng))
        L_ = lanes(lo, hi)
        row = {"lockstep": lockstep(L_)}
        for K in (1, 2, 3):
            for th in (1, 8, 32):
                row[(K, th)] = uniform(L_, K, th)
        res.append(row)
    base = statistics.mean(9 * r["lockstep"] for r in res)
    out = {"blocks_simulated": blocks, "lockstep_steps": statistics.mean(r["lockstep"] for r in res),
           "lockstep_products_per_lane": base, "uniform": []}
    for K in (1, 2, 3):
        for th in (1, 8, 32):
            e = statistics.mean(r[(K, th)][0] for r in res)
            b = statistics.mean(r[(K, th)][1] for r in res)
            out["uniform"].append({"fifo_slots": K, "lds_bytes_per_wave_extra": K * 160 * 64, "thresh": th,
                                   "entry_steps": e, "boundary_steps": b, "products_per_lane": 7 * e + 9 * b,
                                   "ratio_to_lockstep": (7 * e + 9 * b) / base})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8)
