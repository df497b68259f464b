"""The work counters of the long-sequence and live sweeps (gs_sweep_long.hip,
gs_sweep_live.hip), restated on the CPU: the 16 pools
(XCD blockIdx % 8 x half (blockIdx / 8) & 1) split the rank's targets (tiles) in
proportion to their wavefronts, a wavefront's first batch (pair of batches) is its
rank in its pool, every next one comes from the pool's counter.  Whatever order the
counters hand them out in, every batch of every pool is swept exactly once and no
target outside [0, n_local) is touched -- for every grid the launchers produce,
including grids smaller than 16 workgroups (empty pools) and empty shards.  Also the
general sweep's protein path (gs_sweep.hip kDyn): each workgroup's wavefronts share its
range by units of G sequences through an LDS counter."""
import itertools

import pytest

K_REPL = 8


def pools(grid, nwv, n):
    """[(first, count, waves, block ranks)] of the 16 pools (the kernels' arithmetic)."""
    nwaves = grid * nwv
    qn, rn = n // nwaves, n % nwaves
    q8, r8 = grid // K_REPL, grid % K_REPL
    out = []
    for xcd, half in itertools.product(range(K_REPL), range(2)):
        nbx = q8 + (1 if xcd < r8 else 0)
        r0 = xcd * q8 + min(xcd, r8) + ((nbx + 1) >> 1 if half else 0)
        rc = nbx >> 1 if half else (nbx + 1) >> 1
        lw0, lw1 = r0 * nwv, (r0 + rc) * nwv
        first = lw0 * qn + min(lw0, rn)
        cnt = lw1 * qn + min(lw1, rn) - first
        blocks = [b for b in range(grid) if b % K_REPL == xcd and (b // K_REPL) & 1 == half]
        assert len(blocks) == rc
        out.append((first, cnt, rc * nwv, blocks))
    return out


def sweep_pool(nb, nwp, pairs, order_seed):
    """Batches a pool's wavefronts take: static ranks, then counter values handed out
    in an arbitrary interleaving of the wavefronts (order_seed)."""
    import random
    rnd = random.Random(order_seed)
    taken = []
    ctr = 0
    if pairs:  # long kernel: pair v = batches 2v, 2v + 1; first pair = rank
        live = [w for w in range(nwp) if 2 * w < nb]
        cur = {w: 2 * w for w in live}
        while live:
            w = rnd.choice(live)
            b = cur[w]
            taken.append(b)
            if (b & 1) == 0 and b + 1 < nb:
                cur[w] = b + 1
            else:
                nxt = min(2 * (nwp + ctr), nb)
                ctr += 1
                if nxt < nb:
                    cur[w] = nxt
                else:
                    live.remove(w)
    else:  # live kernel: first tile = rank, then nwp + counter (no counter if nb <= nwp)
        live = [w for w in range(nwp) if w < nb]
        cur = {w: w for w in live}
        while live:
            w = rnd.choice(live)
            taken.append(cur[w])
            if nb > nwp:
                nxt = min(nwp + ctr, nb)
                ctr += 1
            else:
                nxt = nb
            if nxt < nb:
                cur[w] = nxt
            else:
                live.remove(w)
    return taken


GRIDS = [1, 3, 8, 15, 16, 17, 64, 255, 256, 513, 768]


@pytest.mark.parametrize("grid", GRIDS)
@pytest.mark.parametrize("nwv", [2, 4, 8])
def test_pools_partition_the_targets(grid, nwv):
    for n in (0, 1, 7, 1000, 100_000, 1_000_003):
        ps = pools(grid, nwv, n)
        spans = sorted((f, c) for f, c, _, _ in ps if c > 0)
        pos = 0
        for f, c in spans:
            assert f == pos and c > 0
            pos += c
        assert pos == n
        # a pool with targets has wavefronts
        assert all(w > 0 for _, c, w, _ in ps if c > 0)


@pytest.mark.parametrize("pairs,per", [(True, 4), (False, 64)])
@pytest.mark.parametrize("grid,nwv,n", [(768, 4, 100_000), (17, 4, 5_000), (3, 8, 999),
                                        (512, 8, 15_625 * 64), (489, 4, 125_000), (1, 2, 1)])
def test_every_batch_swept_once(pairs, per, grid, nwv, n):
    for first, cnt, nwp, _ in pools(grid, nwv, n):
        nb = (cnt + per - 1) // per
        for seed in range(3):
            taken = sweep_pool(nb, nwp, pairs, seed)
            assert sorted(taken) == list(range(nb))
            # the targets of those batches stay inside the pool's range
            for b in taken:
                lo = first + per * b
                assert first <= lo < first + cnt


def wg_ranges(grid, nwv, n):
    """[(first, count)] of the general sweep's workgroups (gs_sweep.hip kDyn, H = 1):
    logical block lb = XCD-major rank of workgroup b, its range the union of its
    wavefronts' static shares."""
    nwaves = grid * nwv
    qn, rn = n // nwaves, n % nwaves
    q8, r8 = grid // K_REPL, grid % K_REPL
    out = []
    for b in range(grid):
        xcd = b % K_REPL
        lb = xcd * q8 + min(xcd, r8) + b // K_REPL
        w0, w1 = lb * nwv, (lb + 1) * nwv
        first = w0 * qn + min(w0, rn)
        out.append((first, w1 * qn + min(w1, rn) - first))
    return out


def sweep_wg(nunits, nwv, order_seed):
    """Units a workgroup's wavefronts take: wid and wid + waves first, then the LDS
    counter (starting at 2 waves) in an arbitrary interleaving of the wavefronts; a
    wavefront stops at its first unit >= nunits."""
    import random
    rnd = random.Random(order_seed)
    ctr = 2 * nwv
    cur = {w: (w, w + nwv) for w in range(nwv)}
    live = [w for w in range(nwv) if w < nunits]
    taken = []
    while live:
        w = rnd.choice(live)
        cu, nu = cur[w]
        taken.append(cu)
        nn = ctr  # the grab made while cu is swept
        ctr += 1
        if nu < nunits:
            cur[w] = (nu, nn)
        else:
            live.remove(w)
    return taken


@pytest.mark.parametrize("grid,nwv,n,G", [(256, 12, 50_000, 2), (256, 12, 1000, 2), (17, 12, 999, 4),
                                          (3, 8, 5, 2), (1, 12, 0, 2), (256, 6, 50_000, 1)])
def test_workgroup_units_swept_once(grid, nwv, n, G):
    rs = wg_ranges(grid, nwv, n)
    spans = sorted(r for r in rs if r[1] > 0)
    pos = 0
    for f, c in spans:
        assert f == pos
        pos += c
    assert pos == n
    for first, cnt in rs:
        nunits = (cnt + G - 1) // G
        for seed in range(3):
            taken = sweep_wg(nunits, nwv, seed)
            assert sorted(taken) == list(range(nunits))
            # every sequence of the range once, none outside it
            seqs = sorted(first + u * G + g for u in taken for g in range(G) if u * G + g < cnt)
            assert seqs == list(range(first, first + cnt))
