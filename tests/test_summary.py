"""TensorBoard event files (manette_amd/summary.py) — CPU: TFRecord framing with masked CRC32C,
Event / Summary protos, and the reference's summary calls (paac.py:23-31, :65-77, :191-199)."""
import os

import numpy as np

from manette_amd import summary


def test_event_file_roundtrip(tmp_path):
    w = summary.EventWriter(str(tmp_path / 'tf'))
    w.add_scalars(7, [('rl/reward', 21.0), ('rl/episode_length', 3410.0)])
    w.add_text(0, 'text', '{"arch": "NIPS"}')
    w.close()
    ev = summary.read_events(w.path)
    assert ev[0][2] == {'file_version': 'brain.Event:2'}
    assert ev[1][1] == 7 and ev[1][2] == {'rl/reward': 21.0, 'rl/episode_length': 3410.0}
    assert ev[2][1] == 0 and ev[2][2] == {'text': '{"arch": "NIPS"}'}
    assert all(e[0] > 1e9 for e in ev)
    raw = bytearray(open(w.path, 'rb').read())
    raw[-6] ^= 1
    open(w.path, 'wb').write(bytes(raw))
    try:
        summary.read_events(w.path)
        assert False, 'corrupt record accepted'
    except ValueError:
        pass


def test_learner_summaries_follow_reference(tmp_path):
    """Episodes from the reference's own host loop (golden G1: the step, reward and length each
    rl/* scalar was written with) come out at the same steps; log_values fires only past 50
    episodes and on global_step % 500 == 0, with the reference's five statistics."""
    root = os.path.dirname(os.path.abspath(__file__))
    z = np.load(os.path.join(root, 'golden', 'host_loop_figar_r11.npz'))
    df = str(tmp_path) + '/'
    open(df + 'args.json', 'w').write('{"game": "pong"}')
    L = summary.LearnerSummaries(df)
    eps = list(zip(z['episode_step'].tolist(), z['episode_reward'].tolist(), z['episode_length'].tolist()))
    assert eps
    L.episodes(eps)
    vals = [float(x) for x in np.random.RandomState(0).randint(-21, 22, 60)]
    L.log_values(vals[:50], 'rewards_per_episode', 1000)   # not > 50 episodes
    L.log_values(vals, 'rewards_per_episode', 1001)        # not on a multiple of 500
    L.log_values(vals, 'rewards_per_episode', 1500)
    L.close()
    files = os.listdir(df + 'tf')
    assert len(files) == 1 and files[0].startswith('events.out.tfevents.')
    ev = summary.read_events(df + 'tf/' + files[0])
    assert ev[1][1] == 0 and ev[1][2]['text'] == '{"game": "pong"}'
    got = [(s, v['rl/reward'], v['rl/episode_length']) for _, s, v in ev if 'rl/reward' in v]
    assert got == [(s, np.float32(r), np.float32(l)) for s, r, l in eps]
    stats = [(s, v) for _, s, v in ev if 'rewards_per_episode/mean' in v]
    assert len(stats) == 1 and stats[0][0] == 1500
    last = np.array(vals[-50:])
    v = stats[0][1]
    assert v['rewards_per_episode/mean'] == np.float32(last.mean())
    assert v['rewards_per_episode/min'] == np.float32(last.min())
    assert v['rewards_per_episode/max'] == np.float32(last.max())
    assert v['rewards_per_episode/std'] == np.float32(last.std())
    assert v['rewards_per_episode/std_over_mean'] == np.float32(min(2, abs(last.std() / last.mean())))


def test_dp_episode_records_merge_in_global_step_order():
    """Data parallel summaries: the chief logs the union of the ranks' episodes in the order
    one process owning every env would have finished them (by their global step, paac.py:184-199)."""
    from manette_amd.paac import merge_episode_records
    r0 = [(17, 1.0, 40), (33, -1.0, 12)]
    r1 = [(21, 0.0, 7), (29, 2.0, 9), (41, 1.0, 3)]
    got = merge_episode_records([r0, r1])
    assert [g for g, _, _ in got] == [17, 21, 29, 33, 41]
    assert got[1] == (21, 0.0, 7) and got[3] == (33, -1.0, 12)
    assert merge_episode_records([[], []]) == []
