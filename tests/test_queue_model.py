"""CPU model of the batch kernels' stream queue and intra-region help protocol (tests/queue_model.py,
DESIGN.md §2.1c): randomized wave interleavings over the launch geometries, the invariants the GPU
tests read from counters, and the two protocol bugs of rounds 4-5 re-introduced as mutations.

The reference has no failure mode here -- NextSplitPoint has no error channel
(repo/splitter/splitter.go:25) -- so a stranded stream would be a failed snapshot: every launch of
the model must finish every stream exactly once with the expected cuts."""
from collections import Counter

import pytest

import queue_model as qm

SEEDS = 150
PATHS = {"claim_ok", "claim_failed", "help_cas_lost", "help_posted", "help_closed", "help_wait_cand",
         "help_wait_none", "help_wait_pending", "help_params_stale", "switch_entry_ready",
         "switch_entry_polled", "yield", "yield_tomb", "tombstone_taken", "late_requeue", "steal",
         "requeued_first_ticket"}
WINDOW_PATHS = {"help_window_next", "help_window_passed"}


@pytest.mark.parametrize("kind", ["buz", "rk"])
def test_protocol_invariants_hold(kind):
    paths = Counter()
    for seed in range(SEEDS):
        L = qm.random_launch(seed, kind)
        v = L.check()
        assert not v, (seed, kind, v[:5])
        paths.update(L.paths)
    # every protocol path was exercised, so the invariants above covered it
    missing = PATHS - {k for k, c in paths.items() if c}
    assert not missing, missing


@pytest.mark.parametrize("kind,window", [("buz", 3), ("buz", 4), ("rk", 4)])
def test_help_windows_keep_the_invariants(kind, window):
    """Regions published a few tiles at a time (BatchArgs::help_window, both batch kernels): the owner
    re-publishes when it passes a window's end or its helpers hold the window's rest without a
    candidate; every stream still finishes once with the expected cuts."""
    paths = Counter()
    for seed in range(SEEDS):
        L = qm.random_launch(seed, kind, window=window)
        v = L.check()
        assert not v, (seed, window, v[:5])
        paths.update(L.paths)
    missing = (PATHS | WINDOW_PATHS) - {"requeued_first_ticket", "steal"} - {k for k, c in paths.items() if c}
    assert not missing, missing


def test_budget_help_mutation_is_caught():
    """Round 5's orphaned ring entries: budget_out without !is_help (kcdc_kernels.hip budget_out in
    split_batch_pipe_kernel) reserves entries a help tile never writes."""
    bad = [s for s in range(100) if qm.random_launch(s, "buz" if s % 2 else "rk", (qm.MUT_BUDGET_HELP,)).check()]
    assert len(bad) >= 5, bad
    v = qm.random_launch(bad[0], "buz" if bad[0] % 2 else "rk", (qm.MUT_BUDGET_HELP,)).check()
    assert any("never written" in x or "tickets - entries" in x for x in v), v


def test_held_register_mutation_is_caught():
    """Round 4's lost tickets: the help task's end took its ticket from a register copy that, on the
    owner-closed path, still held the argument of the take that returned the task (the gfx950
    miscompile).  held_get reads memory's copy instead."""
    bad = [s for s in range(100) if qm.random_launch(s, "buz" if s % 2 else "rk", (qm.MUT_HELD_REGISTER,)).check()]
    assert len(bad) >= 5, bad
    v = qm.random_launch(bad[0], "buz" if bad[0] % 2 else "rk", (qm.MUT_HELD_REGISTER,)).check()
    assert any("dropped" in x or "while holding" in x or "finished" in x for x in v), v


def test_model_expected_cuts_follow_the_chunk_rule():
    """The model's expected tokens: a region's cut is its first candidate tile, else forced."""
    import random
    st = qm.make_streams(random.Random(7), 50, 4, 9)
    for s in st:
        exp = s.expected()
        assert len(exp) == len(s.regions) + (1 if s.end_tail else 0)
        for r, reg in enumerate(s.regions):
            f = reg.first()
            assert exp[r] == (("C", r, f) if f is not None else ("F", r))
