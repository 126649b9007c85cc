"""Scripted bots (script.py:6-83) and game logs (core.py:413-443) against the
reference's own outputs.  CPU only, except the last test (GPU single-game
play written as a log)."""
import gzip
import os
import tempfile

import numpy as np
import pytest

from astro_amd import bots, logs
from astro_amd.core import roll_ships
from tests import golden_io as gio
from tests.test_oracle_golden import _state_from_row

CFG = gio.configs()


def test_scriptbot_decisions_match_reference():
    """ScriptBot's control for every golden input state and every ship's ego
    view == the reference ScriptBot's (tests/golden/script_controls.npz)."""
    tr = gio.Transitions('steps.npz')
    want = gio.load('script_controls.npz')['control']
    made = {}
    for i in range(tr.n):
        name = tr.cfg_names[tr.z['cfg'][i]]
        bot = made.setdefault(name, bots.ScriptBot.create(CFG[name]))
        S = int(tr.z['nships'][i])
        st = _state_from_row(tr, i, S)
        for k in range(S):
            assert bot(roll_ships(st, k)) == want[i, k], (i, k)
    assert bots.NothingBot()(None) == 2


def _golden_log_text():
    with gzip.open(os.path.join(gio.GOLDEN, 'log_short_nothing.jsonl.gz'), 'rt') as f:
        return f.read()


def test_log_round_trip_matches_reference_text():
    """load_log reads a log the reference wrote; save_log writes it back
    byte for byte (core.py:413-443, util.py:13-64)."""
    text = _golden_log_text()
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, 'ref.jsonl')
        open(src, 'w').write(text)
        game = logs.load_log(src)
        assert game.winner is None and len(game.ticks) == 150
        assert game.config == CFG['short']._replace(seed=42)
        dst = os.path.join(d, 'sub', 'again.jsonl')
        logs.save_log(dst, game)
        assert open(dst).read() == text


def test_log_replays_under_the_oracle():
    """The logged controls, replayed through the single-game CPU port from the
    logged first state, reproduce every logged state (the log is a faithful
    trajectory of the physics)."""
    from oracle import port
    text = _golden_log_text()
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, 'ref.jsonl')
        open(src, 'w').write(text)
        game = logs.load_log(src)
    g = port.Game(game.config)
    st = g.create()
    for k, tick in enumerate(game.ticks):
        s = tick.state
        assert np.array_equal(st.ships.x, s.ships.x) and np.array_equal(st.ships.b, s.ships.b), k
        assert np.array_equal(st.bullets.x, s.bullets.x.reshape(-1, 2)), k
        st, reward = g.step(st, tick.control)
        assert np.array_equal(reward, tick.reward), k
    assert st is None


@pytest.mark.gpu
def test_gpu_play_writes_the_reference_log():
    """astro_amd.core.play (the HIP kernel behind the reference's
    create/step surface) with two NothingBots writes the same log as the
    reference's core.play + save_log."""
    from astro_amd import core
    game = core.play(CFG['short']._replace(seed=42), [bots.NothingBot(), bots.NothingBot()])
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, 'gpu.jsonl')
        logs.save_log(path, game)
        assert open(path).read() == _golden_log_text()
