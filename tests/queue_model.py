"""Step-level CPU model of the batch kernels' stream queue and intra-region help protocol.

Test infrastructure only (tests/test_queue_model.py): nothing in the product imports it.

It restates, wave by wave, the state machine that `split_batch_pipe_kernel` (buzhash) and
`split_batch_rk_kernel` (Rabin-Karp) in kopia_amd/csrc/kcdc_kernels.hip run over the shared
queue and help memory, at the granularity at which other waves can observe it: every global
memory operation (the {head, tail} ticket atomic, ring-entry writes and reads, the done counter,
the workgroup flags, the help slots' claim words, granules, result rows, bitmap and held-ticket
words) is one scheduling point, and a seeded scheduler interleaves the waves at random.  What a
tile *scans* is abstracted to data: every stream is a list of regions, every region a list of
tiles that do or do not hold a candidate (and, for help sub-tiles, in which half), so the cut a
wave emits is a token ('C', region, tile) / ('F', region) / ('END',) whose expected list is
known in advance.

Sources it follows (function names; line numbers as of round 6):
  init_ring_kernel (~2624): head = min(n, waves), tail = n, entries 0..n-1, counts failed
  first_ticket, try_steal (~979-1032): preassigned first tickets; requeue of a workgroup that
      has not started
  presolve (~1291-1338): poll the held ticket's entry, done-counter progress + spin cap,
      steal scans, help_find every kHelpEvery polls
  help_publish / help_close / help_find / help_post / help_wait / held_put / held_get
      (~1095-1281)
  the per-tile body of split_batch_pipe_kernel (~1555-1849) and split_batch_rk_kernel
      (~2300-2620): publish, owner claims, budget_out / ends_nocand / switching / reserve, the
      ticket taken at the visit's last tile, the late entry reservation, help tasks (two
      sub-tiles, post or close check), help_wait's three outcomes, requeue by reservation, by a
      late take (a candidate kept the stream alive) or a tombstone, and the switch.

The invariants checked after each launch (check_launch) are the ones the GPU tests measure with
counters (tests/test_gpu_help.py): every stream finished exactly once with the expected cuts,
tickets - entries in {W - 1, W}, no held ticket dropped, every reserved entry written.

Two mutations re-introduce the protocol bugs of rounds 4 and 5:
  MUT_BUDGET_HELP   budget_out without `!is_help`: a help tile of a wave whose last own visit spent
                    its budget reserves a ring entry nobody writes;
  MUT_HELD_REGISTER the help task's end takes its ticket from the register copy, and on the
                    "owner closed the region" path that copy is the stale argument of the take
                    that returned the help task (the gfx950 miscompile).
"""
import random
from collections import Counter
from dataclasses import dataclass
from typing import List, Optional

NONE = 0xFFFFFFFF
TOMB = "tomb"
CLOSED = 1 << 23          # kHelpClosed
HELP_TILES = 128          # kHelpTiles
MUT_BUDGET_HELP = "budget_help"
MUT_HELD_REGISTER = "held_register"


@dataclass
class Region:
    cand: List[bool]                 # per tile: the tile holds a candidate of this region
    half: List[int]                  # per tile with a candidate: its first candidate's sub-tile (0/1)
    forced_ends: bool                # a forced cut at this region's end would finish the stream
    tail_seed: int = 0               # draws the last tile's step count (seeded, not address-based)

    @property
    def K(self):
        return len(self.cand)

    def first(self):
        for i, c in enumerate(self.cand):
            if c:
                return i
        return None


@dataclass
class Stream:
    regions: List[Region]
    end_tail: bool                   # the stream's tail after its last region is cut at n ('END')

    def expected(self):
        out = []
        for r, reg in enumerate(self.regions):
            f = reg.first()
            out.append(("C", r, f) if f is not None else ("F", r))
        if self.end_tail:
            out.append(("END",))
        return out


def make_streams(rng, n, max_regions, max_tiles):
    """Random streams consistent with the kernels' geometry: a region without a candidate ends in
    a forced cut, which finishes the stream only at its last region; a region whose only
    candidates sit in its last tile may have a forced cut that would have ended the stream (the
    "candidate kept the stream alive" path)."""
    out = []
    for _ in range(n):
        R = rng.randrange(0, max_regions + 1)
        regs = []
        for r in range(R):
            K = rng.choice([1, 1, 2, 3, 4, 5, 7, max_tiles])
            p = rng.choice([0.0, 0.1, 0.3, 0.6])
            cand = [rng.random() < p for _ in range(K)]
            half = [rng.randrange(2) for _ in range(K)]
            f = next((i for i, c in enumerate(cand) if c), None)
            last = r == R - 1
            if f is None:
                fe = last
            elif f == K - 1:
                fe = rng.random() < 0.5 and (not last or rng.random() < 0.5)
            else:
                fe = False
            if f is None and not last:
                fe = False
            regs.append(Region(cand, half, fe, rng.randrange(1 << 30)))
        out.append(Stream(regs, rng.random() < 0.7))
    return out


@dataclass
class PStream:
    """The wave's `cur` (kcdc_kernels.hip struct PStream): an own stream or a help task."""
    sid: int
    help: bool = False
    r: int = 0                       # own: region index (s)
    ti: Optional[int] = None         # own: next tile of the region (ct; None = not set up)
    cnt: int = 0                     # own: cuts emitted; help: the published tile index
    cap: int = 0                     # help: the held ticket (register copy)
    cb: int = 0                      # help: the owner's slot
    epoch: int = 0                   # help: the owner slot's epoch
    tile: int = 0                    # help: the region tile it scans
    sub: int = 0                     # help: sub-tile (kHelpSplit = 2)


class Launch:
    def __init__(self, streams, grid, wg_waves, *, kind="buz", help_on=True, quantum=3, min_tiles=3,
                 gap=1, help_every=2, wait_polls=20, spin_cap=4000, steal_spins=16, nb_full=3,
                 delayed_wgs=(), delay_steps=0, mutations=(), seed=0, window=0):
        self.st = streams
        self.n = len(streams)
        self.grid, self.wg_waves = grid, wg_waves
        self.W = grid * wg_waves
        self.kind = kind
        self.help_on = help_on
        self.quantum, self.min_tiles, self.gap = quantum, min_tiles, gap
        self.window = window                       # help windows (BatchArgs::help_window)
        self.help_every, self.wait_polls = help_every, wait_polls
        self.spin_cap, self.steal_spins, self.nb_full = spin_cap, steal_spins, nb_full
        self.mut = set(mutations)
        self.rng = random.Random(seed)
        self.delayed = set(delayed_wgs)
        self.delay_steps = delay_steps
        # ---- memory after init_ring_kernel
        self.head = min(self.W, self.n)
        self.tail = self.n
        self.ring = {e: ("own", PStream(e)) for e in range(self.n)}   # tag e + 1 implied by the key
        self.written = set(range(self.n))
        self.done = 0
        self.err = 0
        self.counts = [None] * self.n
        self.cuts = [[] for _ in range(self.n)]
        self.finished = [0] * self.n
        self.flags = [0] * grid
        self.claim = [(0, 0, 0)] * self.W          # {epoch | top | bottom}
        self.params = [None] * self.W              # (epoch, sid, r, tile0, K)
        self.rows = [[0] * HELP_TILES for _ in range(self.W)]   # (epoch << 40) | (state << 32) | tile
        self.bits = set()
        self.held = [None] * self.W
        # ---- model bookkeeping (not kernel state)
        self.taken = {}                            # ticket -> wave
        self.resolved = set()
        self.exit_ticket = {}                      # wave -> ticket polled when it exited
        self.violations = []
        self.helps = 0
        self.steps = 0
        self.paths = Counter()                     # protocol paths taken (coverage)

    # ------------------------------------------------------------------ helpers
    def cand_in(self, sid, r, tile):
        return self.st[sid].regions[r].cand[tile]

    def nb_of(self, reg, ti):  # steps of a tile: full tiles nb_full, a region's last tile shorter
        if ti == reg.K - 1:
            return 1 + (reg.tail_seed % self.nb_full)
        return self.nb_full

    def emit(self, cur, tok):
        self.cuts[cur.sid].append(tok)
        cur.cnt += 1

    def pstream_region(self, cur):
        """Set up the next region (kcdc_kernels.hip pstream_region); False when finished."""
        if cur.ti is not None:
            return True
        regs = self.st[cur.sid].regions
        if cur.r >= len(regs):
            if self.st[cur.sid].end_tail and (not self.cuts[cur.sid] or self.cuts[cur.sid][-1] != ("END",)):
                self.emit(cur, ("END",))
            return False
        cur.ti = 0
        return True

    def finish(self, cur):
        self.counts[cur.sid] = cur.cnt
        self.finished[cur.sid] += 1
        self.done += 1

    def quantum_of(self, backlog):
        return 1 << 62 if backlog <= 0 else self.quantum

    def take_fresh(self, w):
        t = self.head
        self.head += 1
        if t in self.taken:
            self.violations.append(f"ticket {t} taken twice")
        self.taken[t] = w
        return t, self.tail

    def reserve(self, k=1):
        e = self.tail
        self.tail += k
        return e

    def pwrite(self, e, cur, tomb):
        if e in self.written:
            self.violations.append(f"entry {e} written twice")
        if e >= self.tail:
            self.violations.append(f"entry {e} written but never reserved")
        self.written.add(e)
        self.ring[e] = (TOMB, None) if tomb else ("own", PStream(cur.sid, r=cur.r, ti=cur.ti, cnt=cur.cnt))

    # ------------------------------------------------------------------ help slots
    def help_publish(self, me, ep, cur, K):
        for k in range(K):
            self.rows[me][k] = 0
        self.params[me] = (ep, cur.sid, cur.r, cur.ti, K)
        yield
        self.claim[me] = (ep, K, 1)
        yield
        self.bits.add(me)

    def help_close(self, me, ep):
        self.claim[me] = (ep | CLOSED, 0, 0)
        yield
        self.bits.discard(me)

    def help_find(self, me, w):
        """A waiting wave claims the top tile of the open region with the most unclaimed tiles."""
        slots = sorted(self.bits - {me})
        if not slots:
            return None
        yield
        # one bitmap word per lane, one set bit per word (rotated): a random subset of slots
        words = {}
        for g in slots:
            words.setdefault(g >> 5, []).append(g)
        cand = [self.rng.choice(v) for v in words.values()]
        best, bg, bw = 0, None, None
        for g in cand:
            ep, top, bot = self.claim[g]
            if ep != 0 and not (ep & CLOSED) and top >= bot + self.gap:
                key = (top - bot) * 64 + self.rng.randrange(64)
                if key > best:
                    best, bg, bw = key, g, (ep, top, bot)
        yield
        if bg is None:
            return None
        if self.claim[bg] != bw:                   # compare-and-swap lost the race
            self.paths["help_cas_lost"] += 1
            return None
        ep, top, bot = bw
        self.claim[bg] = (ep, top - 1, bot)
        k = top - 1
        yield
        p = self.params[bg]
        if p is None or p[0] != ep:                # the owner has moved on: nobody waits for this tile
            self.paths["help_params_stale"] += 1
            return None
        _, sid, r, tile0, K = p
        return PStream(sid, help=True, r=r, cnt=k, cb=bg, epoch=ep, tile=tile0 + k, sub=0)

    def help_post(self, g, ep, k, tile):
        v = (ep << 40) | ((2 << 32) | tile if tile is not None else (1 << 32))
        self.rows[g][k] = max(self.rows[g][k], v)
        self.helps += 1
        yield

    def help_wait(self, me, ep, k0, K, tile0):
        """Owner whose claim failed: first candidate tile among [k0, K) (region tile), -1 none,
        or -2 - k for a tile still pending after the wait bound."""
        polls = 0
        while True:
            res, pend = -1, None
            for k in range(k0, K):
                v = self.rows[me][k]
                mine = (v >> 40) == ep
                stt = (v >> 32) & 0xFF if mine else 0
                if stt == 2:
                    res = v & 0xFFFFFFFF
                    break
                if stt != 1:
                    pend = k
                    break
            yield
            if pend is None:
                self.paths["help_wait_cand" if res >= 0 else "help_wait_none"] += 1
                return res
            polls += 1
            if polls > self.wait_polls:
                self.paths["help_wait_pending"] += 1
                return -2 - pend

    # ------------------------------------------------------------------ queue
    def try_steal(self, w):
        found = next((b for b in range(self.grid) if self.flags[b] == 0), None)
        yield
        if found is None:
            return
        if self.flags[found] != 0:
            return
        self.flags[found] = 2
        self.paths["steal"] += 1
        yield
        sids = [v * self.grid + found for v in range(self.wg_waves) if v * self.grid + found < self.n]
        if not sids:
            return
        e0 = self.reserve(len(sids))
        yield
        for i, sid in enumerate(sids):
            self.pwrite(e0 + i, PStream(sid), False)
            yield

    def presolve(self, w, t, me, can_help):
        """0 stop, 1 resolved (cur in w.cur), 2 tombstone, 3 help task."""
        idle, seen = 0, None
        spin = 0
        while True:
            ent = self.ring.get(t) if t in self.written else None
            yield
            if ent is not None:
                self.resolved.add(t)
                if ent[0] == TOMB:
                    return 2
                src = ent[1]
                w.cur = PStream(src.sid, r=src.r, ti=src.ti, cnt=src.cnt)
                return 1
            stop = False
            if spin % 4 == 0:                      # kDoneEvery
                d = self.done
                yield
                idle = idle + 1 if d == seen else 0
                seen = d
                if d >= self.n:
                    stop = True
                elif idle + 1 >= self.spin_cap:
                    self.err += 1
                    stop = True
            if stop:
                self.exit_ticket[w.id] = t
                return 0
            if self.steal_spins and spin % self.steal_spins == self.steal_spins - 1:
                yield from self.try_steal(w)
                spin += 1
                continue
            if can_help and spin % self.help_every == self.help_every - 1:
                task = yield from self.help_find(me, w)
                if task is not None:
                    w.cur = task
                    return 3
            yield
            spin += 1

    # ------------------------------------------------------------------ one wave
    def wave(self, w):
        me = w.id
        block, widx = me % self.grid, me // self.grid
        # the workgroup flag: 0 -> 1 (ours), or 2 (requeued by a stealer before we started)
        old = self.flags[block]
        if old == 0:
            self.flags[block] = 1
        yield
        t0 = widx * self.grid + block
        take_t = t0 if t0 < self.n else NONE
        if t0 < self.n:
            self.taken[t0] = me
        take_backlog = self.n - self.W
        take_claim = (old & 3) if t0 < self.n else NONE
        budget = 1 << 62
        hep, hs_pub, hs_k, hs_tile, hs_needpub, hs_helped = 0, False, 0, 0, True, False
        need_take = True
        while True:
            if need_take:
                # ---------------- take_blocking
                t, backlog_hint, claim = take_t, take_backlog, take_claim
                got = False
                while True:
                    backlog = backlog_hint
                    if t == NONE:
                        if w.holding is not None:
                            self.violations.append(f"wave {me} took a fresh ticket while holding {w.holding}")
                        t, tl = self.take_fresh(me)
                        backlog = tl - t - 1
                        yield
                    held = t
                    w.holding = held
                    r = yield from self.presolve(w, held, me, self.help_on and claim == NONE)
                    if r == 0:
                        return
                    if r == 3:
                        self.held[me] = held           # held_put
                        yield
                        w.cur.cap = held
                        w.stale_take_arg = take_t      # what the register held before the take
                        got = True
                        break
                    w.holding = None
                    t = NONE
                    if claim != NONE:
                        requeued = claim == 2
                        claim = NONE
                        if requeued:
                            self.paths["requeued_first_ticket"] += 1
                            continue
                    if r == 2:
                        self.paths["tombstone_taken"] += 1
                        continue
                    budget = self.quantum_of(backlog)
                    if self.pstream_region(w.cur):
                        got = True
                        break
                    self.finish(w.cur)
                    yield
                need_take = False
                hs_needpub = True
            cur = w.cur
            is_help = cur.help
            if is_help:
                reg = self.st[cur.sid].regions[cur.r]
                last_of_region = cur.sub == 1 or self.nb_of(reg, cur.tile) == 1
                nb = 1
            else:
                reg = self.st[cur.sid].regions[cur.r]
                last_of_region = cur.ti == reg.K - 1
                nb = self.nb_of(reg, cur.ti)
            # a region new to this wave: publish it when it is long enough to share
            if hs_needpub and not is_help:
                K = reg.K - cur.ti
                hs_pub, hs_k, hs_tile, hs_needpub, hs_helped = False, 0, 0, False, False
                if self.help_on and self.min_tiles <= K <= HELP_TILES:
                    Kw = min(K, self.window) if self.window else K   # a window of the region
                    hep += 1
                    hs_pub, hs_k = True, Kw
                    yield from self.help_publish(me, hep, cur, Kw)
            claim_next_r = hs_pub and not is_help and not last_of_region and hs_tile + 1 < hs_k
            if MUT_BUDGET_HELP in self.mut:
                budget_out = not hs_helped and budget - 1 <= 0
            else:
                budget_out = not is_help and not hs_helped and budget - 1 <= 0
            ends_nocand = (not is_help) and last_of_region and reg.forced_ends
            switching = not is_help and (budget_out or ends_nocand)
            reserve = budget_out and not ends_nocand
            claim_next = claim_next_r and not switching
            tk, nbacklog = None, 0
            if switching:
                if w.holding is not None:
                    self.violations.append(f"wave {me} took a fresh ticket while holding {w.holding}")
                tk, tl = self.take_fresh(me)
                nbacklog = tl + (1 if reserve else 0) - tk - 1
                yield
            # ---------------- the tile's steps
            pe = None
            claim_ok, claim_known = False, not claim_next
            claim_word = None
            ev = None
            poll_step = nb // 2 if nb > 1 else 0
            hit_tile = None
            for s in range(nb):
                if self.kind == "buz":
                    if claim_next and s >= 2 and s == nb - 1 and claim_word is not None:
                        claim_ok, claim_known, hs_helped = self._decode(claim_word, hep, hs_k, hs_helped)
                    if reserve and s == nb - 1:
                        pe = self.reserve()
                        yield
                    if switching and s == poll_step:
                        ev = self.ring.get(tk) if tk in self.written else None
                        yield
                    if claim_next and s == 1:
                        claim_word = self.claim[me]       # help_claim_dma: read back a step later
                        yield
                    if claim_next and s == 0:
                        ep, top, bot = self.claim[me]
                        self.claim[me] = (ep, top, bot + 1)
                        yield
                else:  # rk: the claim's own return value is decoded at fill 2; refill_last at the end
                    if claim_next and s == 0:
                        ep, top, bot = self.claim[me]
                        self.claim[me] = (ep, top, bot + 1)
                        claim_word = self.claim[me]
                        yield
                    if claim_next and s == 1:
                        claim_ok, claim_known, hs_helped = self._decode(claim_word, hep, hs_k, hs_helped)
                    if s == nb - 1:
                        if reserve:
                            pe = self.reserve()
                            yield
                        if switching:
                            ev = self.ring.get(tk) if tk in self.written else None
                            yield
                yield                                    # the step's hashing
            # ---------------- end of tile
            if not claim_known:
                if self.kind == "buz" and nb != 2:
                    claim_word = self.claim[me]
                    yield
                claim_ok, claim_known, hs_helped = self._decode(claim_word, hep, hs_k, hs_helped)
            if reserve and pe is None:
                pe = self.reserve()
                yield
            if is_help:
                one_sub = self.nb_of(reg, cur.tile) == 1     # a short tile: one sub-tile
                has = reg.cand[cur.tile] and (one_sub or reg.half[cur.tile] == cur.sub)
                done = True
                if has or last_of_region:
                    yield from self.help_post(cur.cb, cur.epoch, cur.cnt, cur.tile if has else None)
                else:
                    ep = self.claim[cur.cb][0]
                    yield
                    done = ep != cur.epoch
                if not done:
                    cur.sub += 1
                    continue
                need_take = True
                path = "posted" if (has or last_of_region) else "closed"
                self.paths["help_" + path] += 1
                if MUT_HELD_REGISTER in self.mut and path == "closed":
                    take_t = w.stale_take_arg           # the miscompiled flow block: no copy on this path
                elif MUT_HELD_REGISTER in self.mut:
                    take_t = cur.cap
                else:
                    take_t = self.held[me]              # held_get: memory's copy
                    if take_t != cur.cap:
                        self.violations.append("held ticket audit mismatch")
                    yield
                take_backlog, take_claim = 0, NONE
                continue
            region_changed = True
            cut = None
            if reg.cand[cur.ti]:
                cut = ("C", cur.r, cur.ti)
            elif last_of_region:
                cut = ("F", cur.r)
            elif claim_next and not claim_ok:
                tile0 = cur.ti - hs_tile
                res = yield from self.help_wait(me, hep, hs_tile + 1, hs_k, tile0)
                if res >= 0:
                    cut = ("C", cur.r, res)
                elif res == -1 and tile0 + hs_k < reg.K:   # no candidate in the window: the next one
                    self.paths["help_window_next"] += 1
                    cur.ti = tile0 + hs_k
                    yield from self.help_close(me, hep)
                    hs_pub, hs_k, hs_tile, hs_needpub, hs_helped = False, 0, 0, True, False
                    region_changed = False
                elif res == -1:
                    cut = ("F", cur.r)
                else:
                    cur.ti = tile0 + (-2 - res)
                    yield from self.help_close(me, hep)
                    hs_pub, hs_k, hs_tile, hs_needpub, hs_helped = False, 0, 0, False, False
                    region_changed = False
            else:
                cur.ti += 1
                hs_tile += 1
                budget -= 1
                region_changed = False
                if hs_pub and hs_tile >= hs_k:            # past its published window: the next one
                    self.paths["help_window_passed"] += 1
                    yield from self.help_close(me, hep)
                    hs_pub, hs_k, hs_tile, hs_needpub, hs_helped = False, 0, 0, True, False
            if cut is not None:
                self.emit(cur, cut)
                cur.r += 1
                cur.ti = None
            if region_changed:
                if hs_pub:
                    yield from self.help_close(me, hep)
                hs_pub, hs_k, hs_tile, hs_needpub, hs_helped = False, 0, 0, True, False
            live = self.pstream_region(cur)
            if not live:
                self.finish(cur)
                yield
            if not switching and live:
                continue
            if hs_pub:
                yield from self.help_close(me, hep)
            hs_pub, hs_k, hs_tile, hs_needpub, hs_helped = False, 0, 0, True, False
            if reserve:
                self.paths["yield_tomb" if not live else "yield"] += 1
                self.pwrite(pe, cur, not live)
                yield
            elif live:
                self.paths["late_requeue"] += 1
                e = self.reserve()
                yield
                self.pwrite(e, cur, False)
                yield
            if switching:
                w.holding = tk                           # (an entry not yet landed is polled by the take)
            if switching:
                self.paths["switch_entry_ready" if ev is not None else "switch_entry_polled"] += 1
            if ev is not None and ev[0] != TOMB:
                self.resolved.add(tk)
                w.holding = None
                src = ev[1]
                w.cur = PStream(src.sid, r=src.r, ti=src.ti, cnt=src.cnt)
                budget = self.quantum_of(nbacklog)
                if self.pstream_region(w.cur):
                    continue
                self.finish(w.cur)
                yield
                need_take, take_t, take_backlog, take_claim = True, NONE, 0, NONE
                continue
            need_take = True
            take_t = tk if switching else NONE
            take_backlog = nbacklog
            take_claim = NONE

    def _decode(self, cw, hep, K, helped):
        ep, top, bot = cw
        ok = ep == hep and bot <= top
        self.paths["claim_ok" if ok else "claim_failed"] += 1
        if top < K:
            helped = True
        return ok, True, helped

    # ------------------------------------------------------------------ scheduler
    def run(self, max_steps=3_000_000):
        @dataclass
        class W:
            id: int
            cur: Optional[PStream] = None
            holding: Optional[int] = None
            stale_take_arg: int = NONE

        waves = [W(i) for i in range(self.W)]
        gens = {w.id: self.wave(w) for w in waves}
        live = list(gens)
        while live:
            self.steps += 1
            if self.steps > max_steps:
                self.violations.append("model did not terminate")
                break
            cand = [i for i in live if (i % self.grid) not in self.delayed or self.steps > self.delay_steps]
            if not cand:
                continue
            i = self.rng.choice(cand)
            try:
                next(gens[i])
            except StopIteration:
                live.remove(i)
        return self

    # ------------------------------------------------------------------ invariants
    def check(self):
        v = list(self.violations)
        for sid, s in enumerate(self.st):
            if self.finished[sid] != 1:
                v.append(f"stream {sid} finished {self.finished[sid]} times")
            elif self.cuts[sid] != s.expected():
                v.append(f"stream {sid} cuts {self.cuts[sid]} != {s.expected()}")
        d = self.head - self.tail
        if d not in (self.W - 1, self.W):
            v.append(f"tickets - entries = {d}, not in {{{self.W - 1}, {self.W}}}")
        unwritten = [e for e in range(self.tail) if e not in self.written]
        if unwritten:
            v.append(f"reserved entries never written: {unwritten[:8]}")
        held_at_exit = set(self.exit_ticket.values())
        dropped = [t for t in self.taken if t not in self.resolved and t not in held_at_exit]
        if dropped:
            v.append(f"held tickets dropped: {sorted(dropped)[:8]}")
        if self.err:
            v.append(f"{self.err} waves gave up")
        return v


def random_launch(seed, kind="buz", mutations=(), window=None):
    """One launch of a random geometry.  The knobs stand for the kernels' geometry parameters:
    grid x waves per workgroup (the persistent grid), streams against waves (fewer than, equal to,
    a few more, many more: the backlog that turns yields on), regions and tiles per stream (the
    average size / lane cap: tiles per region), steps per tile (nb_full: lane cap / 128 B), the
    visit quantum in tiles (KCDC_QUANTUM_TILES), the smallest published region
    (KCDC_HELP_MIN_TILES), the owner's wait bound (KCDC_HELP_WAIT_TICKS), help on or off (the
    per-name policy), a workgroup that starts late (another kernel holds its CU: try_steal), and
    the help window (BatchArgs::help_window: regions published a few tiles at a time; drawn from
    its own generator so the other draws of a seed stay as they were)."""
    rng = random.Random(seed)
    grid = rng.choice([1, 2, 3, 4])
    wgw = rng.choice([2, 4, 8])
    W = grid * wgw
    n = rng.choice([1, W // 2 or 1, W, W + 3, 3 * W, 5 * W])
    streams = make_streams(rng, n, rng.choice([1, 3, 6]), rng.choice([8, 16, 40]))
    delayed = {rng.randrange(grid)} if grid > 1 and rng.random() < 0.3 else set()
    L = Launch(streams, grid, wgw, kind=kind, help_on=rng.random() < 0.85, quantum=rng.choice([1, 2, 3, 6]),
               min_tiles=rng.choice([2, 3]), nb_full=rng.choice([1, 2, 3, 4]), wait_polls=rng.choice([3, 20, 200]),
               delayed_wgs=delayed, delay_steps=rng.choice([100, 2000, 20000]), mutations=mutations, seed=seed,
               window=random.Random(seed ^ 0x5A5A).choice([0, 0, 3, 4, 6]) if window is None else window)
    L.run()
    return L
