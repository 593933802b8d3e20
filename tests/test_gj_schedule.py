"""CPU model of k_gj_persist's task schedule (sparsergps_amd/csrc/k_dense.hip).

The persistent Gauss-Jordan kernel runs the whole m x m SPD inverse in one launch: workgroups
claim tickets in order (interior tiles of a row paired per task) and each task waits on flags
(tile versions, "operands loaded", pivot ready) before it reads or overwrites tiles in place.  This model restates the ticket decoding
and the flag protocol task by task, runs G simulated workgroups under random interleavings
(each wait / load / store is a separate scheduling point), and checks that

* no interleaving deadlocks (a task only waits for smaller tickets), and
* the in-place result equals the inverse (the "loaded" flags keep the column / row tasks from
  overwriting A_ik / A_kj before every interior task of the step has read them), together with
  the pivot log-determinants.

The numerics are numpy's; the GPU kernel's own parity is covered by the -m gpu suites.
"""
import numpy as np
import pytest


def decode(t, nb):
    """k_gj_persist's ticket -> (kind, k, i, js); kinds: pivot0, unit (interior tiles (i, j) for
    j in js: the look-ahead (k+1, k+1) alone, the others paired along their row), col, row,
    diag (js = (j,))."""
    if t == 0:
        return ("pivot0", 0, 0, (0,))
    n1 = nb - 1
    half = (n1 + 1) // 2
    u_reg = 1 + n1 // 2 + (n1 - 1) * half + 2 * n1 + 1
    s = t - 1
    k = min(s // u_reg, n1)
    r = s - k * u_reg
    last = k == n1
    if not last and r == 0:
        return ("unit", k, (k + 1) % nb, ((k + 1) % nb,))
    q = r if last else r - 1
    for a in range(n1):
        skip = 1 if (a == 0 and not last) else 0
        cnt = n1 - skip
        u = (cnt + 1) // 2
        if q < u:
            b0 = skip + 2 * q
            bs = (b0, b0 + 1) if b0 + 1 < n1 else (b0,)
            return ("unit", k, (k + 1 + a) % nb, tuple((k + 1 + b) % nb for b in bs))
        q -= u
    r = q
    if r < 2 * n1:
        col = r < n1
        x = (k + 1 + (r if col else r - n1)) % nb
        return ("col", k, x, (k,)) if col else ("row", k, k, (x,))
    return ("diag", k, k, (k,))


def ntasks(nb):
    n1 = nb - 1
    half = (n1 + 1) // 2
    u_reg = 1 + n1 // 2 + (n1 - 1) * half + 2 * n1 + 1
    return 1 + n1 * u_reg + n1 * half + 2 * n1 + 1


class Chain:
    def __init__(self, A, B=None, beta=0.0):
        self.mp = A.shape[0]
        self.nb = self.mp // 64
        self.src0 = A.copy()
        self.src0b = None if B is None else B.copy()
        self.beta = beta
        # in place (dense_spd_inverse) or into a distinct output (dense_spd_inverse_sum)
        self.buf = self.src0 if B is None else np.full_like(A, np.nan)
        nb = self.nb
        self.ver = np.zeros((nb, nb), int)
        self.loaded = np.zeros((nb, nb), int)
        self.piv = np.zeros(nb, int)
        self.P = [None] * nb
        self.logd = np.zeros(nb)

    def tile(self, k, i, j):
        sl = (slice(64 * i, 64 * i + 64), slice(64 * j, 64 * j + 64))
        if k == 0:
            t = self.src0[sl].copy()
            if self.src0b is not None:
                t = t + self.beta * self.src0b[sl]
            return t
        return self.buf[sl].copy()

    def put(self, i, j, v):
        self.buf[64 * i:64 * i + 64, 64 * j:64 * j + 64] = v

    def pivot(self, k, T):
        self.P[k] = np.linalg.inv(T)
        self.logd[k] = 0.5 * np.linalg.slogdet(T)[1]

    def task(self, t):
        """Generator: yields wait predicates; everything between two yields is atomic."""
        kind, k, i, js = decode(t, self.nb)
        nb = self.nb
        if kind == "pivot0":
            self.pivot(0, self.tile(0, 0, 0))
            self.piv[0] = 1
            return
        if kind == "unit":
            if k > 0:
                yield lambda: min([self.ver[i, k]] + [min(self.ver[i, j], self.ver[k, j])
                                                      for j in js]) >= k
            aik = self.tile(k, i, k)
            ops = [(j, self.tile(k, k, j), self.tile(k, i, j)) for j in js]
            yield None   # the loads land; then "loaded"
            for j in js:
                self.loaded[i, j] = k + 1
            yield lambda: self.piv[k] >= 1
            c = aik @ self.P[k]
            outs = [(j, aij - c @ akj) for j, akj, aij in ops]
            yield None
            if i == k + 1 and js == (k + 1,):
                # the look-ahead: its fresh tile feeds only its own pivot (not stored, no flag;
                # step k+1's (k+1, k+1) task writes P_{k+1} there)
                self.pivot(k + 1, outs[0][1])
                yield None
                self.piv[k + 1] = 1
                return
            for j, v in outs:
                self.put(i, j, v)
            for j, _ in outs:
                self.ver[i, j] = k + 1
            return
        j = js[0]
        if kind in ("col", "row"):
            if k > 0:
                yield lambda: self.ver[i, j] >= k
            a = self.tile(k, i, j)
            yield lambda: self.piv[k] >= 1
            v = -(a @ self.P[k]) if kind == "col" else self.P[k] @ a
            if kind == "col":
                yield lambda: all(self.loaded[i, (k + 1) % nb if q == k else q] >= k + 1
                                  for q in range(nb))
            else:
                yield lambda: all(self.loaded[(k + 1) % nb if q == k else q, j] >= k + 1
                                  for q in range(nb))
            self.put(i, j, v)
            self.ver[i, j] = k + 1
            return
        yield lambda: self.piv[k] >= 1
        self.put(k, k, self.P[k])
        self.ver[k, k] = k + 1


def run(chain, G, rng):
    ntask = ntasks(chain.nb)
    ticket = 0
    workers = [None] * G          # (generator, pending predicate)
    done = [False] * G
    while not all(done):
        ready = []
        for w in range(G):
            if done[w]:
                continue
            if workers[w] is None or workers[w][1] is None or workers[w][1]():
                ready.append(w)
        assert ready, "deadlock: every workgroup waits"
        w = ready[rng.integers(len(ready))]
        if workers[w] is None:
            if ticket >= ntask:
                done[w] = True
                continue
            workers[w] = (chain.task(ticket), None)
            ticket += 1
        gen = workers[w][0]
        try:
            workers[w] = (gen, next(gen))
        except StopIteration:
            workers[w] = None


def spd(mp, rng):
    X = rng.standard_normal((mp, mp + 7))
    return X @ X.T / mp + 0.5 * np.eye(mp)


@pytest.mark.parametrize("nb,G", [(1, 1), (2, 1), (2, 4), (3, 2), (4, 16), (5, 3), (6, 36)])
def test_schedule_inverts_in_place(nb, G):
    rng = np.random.default_rng(nb * 100 + G)
    A = spd(64 * nb, rng)
    for rep in range(3):
        ch = Chain(A)
        run(ch, G, rng)
        np.testing.assert_allclose(ch.buf @ A, np.eye(64 * nb), atol=1e-9)
        assert abs(ch.logd.sum() - 0.5 * np.linalg.slogdet(A)[1]) < 1e-9
        assert (ch.ver == nb).all()   # every tile's last writer in step nb - 1 sets nb


@pytest.mark.parametrize("nb,G", [(1, 2), (3, 4), (4, 7)])
def test_schedule_sum_form(nb, G):
    rng = np.random.default_rng(7 + nb)
    A, B = spd(64 * nb, rng), spd(64 * nb, rng)
    ch = Chain(A, B, 0.3)
    run(ch, G, rng)
    np.testing.assert_allclose(ch.buf @ (A + 0.3 * B), np.eye(64 * nb), atol=1e-9)


def test_decode_covers_every_tile_once_per_step():
    for nb in range(1, 10):
        seen = {}
        for t in range(1, ntasks(nb)):
            kind, k, i, js = decode(t, nb)
            for j in js:
                assert (k, i, j) not in seen
                seen[(k, i, j)] = kind
                assert kind == ("diag" if i == k and j == k else "col" if j == k else
                                "row" if i == k else "unit")
            if kind == "unit" and len(js) == 2:
                assert js[1] == (js[0] + 1) % nb != k
        assert len(seen) == nb ** 3
        # the first task of each step (but the last) is its look-ahead tile, alone
        n1 = nb - 1
        half = (n1 + 1) // 2
        u_reg = 1 + n1 // 2 + (n1 - 1) * half + 2 * n1 + 1
        for k in range(nb - 1):
            assert decode(1 + k * u_reg, nb) == ("unit", k, k + 1, (k + 1,))
