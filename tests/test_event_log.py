"""Event log: the protobuf wire format of the reference's event.proto
and its '=l' framing (event_log.py:48-58, :103-111), checked against google.protobuf
messages built from the same schema, plus the native host writer (cp_eventlog_*,
no GPU needed).  The GPU encoder is checked in tests/test_gpu_event_log.py."""
import ctypes as C
import os
import struct

import numpy as np
import pytest

from cartpoleplusplus_amd import abi, event_log as EL, native

pb = pytest.importorskip("google.protobuf")


@pytest.fixture(scope="module")
def msgs():
    """event.proto:1-35 (package cp, proto2) as dynamic protobuf classes."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="event_test.proto", package="cp", syntax="proto2")

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
    OPT, REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    msg("Render", [("height", 1, F.TYPE_INT32, OPT, None), ("width", 2, F.TYPE_INT32, OPT, None),
                   ("png_bytes", 3, F.TYPE_BYTES, OPT, None)])
    msg("State", [("cart_pose", 1, F.TYPE_FLOAT, REP, None), ("pole_pose", 2, F.TYPE_FLOAT, REP, None),
                  ("render", 3, F.TYPE_MESSAGE, REP, ".cp.Render")])
    msg("Event", [("action", 1, F.TYPE_FLOAT, REP, None), ("state", 2, F.TYPE_MESSAGE, REP, ".cp.State"),
                  ("reward", 3, F.TYPE_FLOAT, OPT, None)])
    msg("Episode", [("event", 1, F.TYPE_MESSAGE, REP, ".cp.Event")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = message_factory.GetMessageClass
    return {n: get(pool.FindMessageTypeByName(f"cp.{n}")) for n in ("Render", "State", "Event", "Episode")}


def _pb_event(msgs, states, action=None, reward=None, renders=None):
    ev = msgs["Event"]()
    if action is not None:
        ev.action.extend(action)
    for st in states:
        s = ev.state.add()
        s.cart_pose.extend(st[0])
        s.pole_pose.extend(st[1])
    if renders:
        for rr in renders:
            s = ev.state.add()
            for (h, w, png) in rr:
                r = s.render.add()
                r.height, r.width, r.png_bytes = h, w, png
    if reward is not None:
        ev.reward = reward
    return ev


def test_lowdim_event_bytes_equal_protobuf(msgs):
    rng = np.random.default_rng(0)
    for R in (1, 2, 3):
        st = rng.standard_normal((R, 2, 7)).astype(np.float32)
        act = rng.uniform(-1, 1, 4).astype(np.float32)
        mine = EL.encode_event([EL.encode_state_lowdim(s[0], s[1]) for s in st], act, 1.0)
        ref = _pb_event(msgs, [(s[0], s[1]) for s in st], act, 1.0).SerializeToString()
        assert mine == ref
        mine0 = EL.encode_event([EL.encode_state_lowdim(s[0], s[1]) for s in st])
        assert mine0 == _pb_event(msgs, [(s[0], s[1]) for s in st]).SerializeToString()


def test_render_event_bytes_equal_protobuf(msgs):
    png = EL.rgb_to_png(np.random.default_rng(1).uniform(0, 1, (5, 7, 3)))
    mine = EL.encode_event([EL.encode_state_renders([(5, 7, png), (5, 7, png)])])
    ref = _pb_event(msgs, [], renders=[[(5, 7, png), (5, 7, png)]]).SerializeToString()
    assert mine == ref


def test_episode_and_framing_parse_with_protobuf(msgs, tmp_path):
    path = str(tmp_path / "ep.log")
    log = EL.EventLog(path, use_raw_pixels=False)
    rng = np.random.default_rng(2)
    episodes = []
    for e in range(3):
        log.reset()
        s0 = rng.standard_normal((2, 2, 7)).astype(np.float32)
        log.add_just_state(s0)
        evs = [(None, s0, None)]
        for t in range(4 + e):
            a = rng.uniform(-1, 1, (1, 2)).astype(np.float32)
            s = rng.standard_normal((2, 2, 7)).astype(np.float32)
            log.add(s, a, 1.0)
            evs.append((a, s, 1.0))
        episodes.append(evs)
    log.reset()                      # the reference writes an episode at the next reset
    raw = open(path, "rb").read()
    pos, got = 0, []
    while pos < len(raw):
        (n,) = struct.unpack("=l", raw[pos:pos + 4])
        ep = msgs["Episode"]()
        ep.ParseFromString(raw[pos + 4:pos + 4 + n])
        got.append(ep)
        pos += 4 + n
    assert len(got) == 3
    for ep, evs in zip(got, episodes):
        assert len(ep.event) == len(evs)
        assert len(ep.event[0].action) == 0 and not ep.event[0].HasField("reward")  # replay_memory.py:51-53
        for pe, (a, s, r) in zip(ep.event, evs):
            np.testing.assert_array_equal(np.array([[st.cart_pose, st.pole_pose] for st in pe.state], np.float32), s)
            if a is not None:
                np.testing.assert_array_equal(np.array(pe.action, np.float32), a.reshape(-1))
                assert pe.reward == r
    # our reader agrees with protobuf
    mine = list(EL.EventLogReader(path).entries())
    assert [len(e.event) for e in mine] == [len(e.event) for e in got]
    np.testing.assert_array_equal(EL.read_state_from_event(mine[1].event[2]), episodes[1][2][1])


def test_pixel_state_round_trip(tmp_path):
    rng = np.random.default_rng(3)
    u8 = rng.integers(0, 256, (6, 5, 3, 2, 3)).astype(np.float64) / 255.0    # (H, W, 3, C, R)
    path = str(tmp_path / "px.log")
    log = EL.EventLog(path, use_raw_pixels=True)
    log.reset()
    log.add_just_state(u8)
    log.add(u8, 2, 1.0)              # a discrete action is logged as one number (event_log.py:87-88)
    log.close()
    ep = next(EL.EventLogReader(path).entries())
    st = EL.read_state_from_event(ep.event[1])
    assert st.shape == (6, 5, 3, 2, 3)
    np.testing.assert_allclose(st, u8, atol=1e-7)
    assert ep.event[1].action == [2.0]


def test_record_sizes_match_encoder():
    lib = native.load()
    rng = np.random.default_rng(4)
    for R in (1, 2, 3, 4):
        st = [EL.encode_state_lowdim(*rng.standard_normal((2, 7))) for _ in range(R)]
        cont = EL.episode_entry(EL.encode_event(st, [0.1, 0.2, 0.3, 0.4], 1.0))
        disc = EL.episode_entry(EL.encode_event(st, [1.0, 3.0], 1.0))
        reset = EL.episode_entry(EL.encode_event(st))
        assert lib.cp_event_record_bytes(abi.CP_ACTION_CONTINUOUS, R, 1) == len(cont)
        assert lib.cp_event_record_bytes(abi.CP_ACTION_DISCRETE, R, 1) == len(disc)
        assert lib.cp_event_record_bytes(abi.CP_ACTION_DISCRETE, R, 0) == len(reset)


def test_native_writer_frames_episodes(msgs, tmp_path):
    """cp_eventlog_write: step records append, a reset record writes the open episode
    and starts the next; close writes what is left."""
    lib = native.load()
    B, R = 3, 2
    rng = np.random.default_rng(5)
    enc = lambda s, a=None, r=None: EL.episode_entry(EL.encode_event(
        [EL.encode_state_lowdim(x[0], x[1]) for x in s], a, r))
    sb, rb = lib.cp_event_record_bytes(0, R, 1), lib.cp_event_record_bytes(0, R, 0)
    path = str(tmp_path / "native.log")
    h = C.c_void_p()
    assert lib.cp_eventlog_open(path.encode(), B, C.byref(h)) == 0
    expect = {i: [] for i in range(B)}
    written = []

    def call(flags, steps, resets):
        sr = np.zeros((B, sb), np.uint8)
        rr = np.zeros((B, rb), np.uint8)
        for i in range(B):
            if flags[i] & 1:
                sr[i] = np.frombuffer(steps[i], np.uint8)
                expect[i].append(steps[i])
            if flags[i] & 2:
                rr[i] = np.frombuffer(resets[i], np.uint8)
                if expect[i]:
                    written.append(b"".join(expect[i]))
                expect[i] = [resets[i]]
        f = np.asarray(flags, np.uint8)
        assert lib.cp_eventlog_write(h, f.ctypes.data, sr.ctypes.data, sb, rr.ctypes.data, rb) == 0

    st = lambda: rng.standard_normal((R, 2, 7)).astype(np.float32)
    call([2, 2, 2], None, [enc(st()) for _ in range(B)])
    for t in range(5):
        fl = [1, 1 | (2 if t == 2 else 0), 1 if t < 3 else 0]
        call(fl, [enc(st(), rng.uniform(-1, 1, 4), 1.0) for _ in range(B)],
             [enc(st()) for _ in range(B)])
    assert lib.cp_eventlog_close(h) == 0
    for i in range(B):
        if expect[i]:
            written.append(b"".join(expect[i]))
    got = [open(path, "rb").read()]
    raw, pos, bodies = got[0], 0, []
    while pos < len(raw):
        (n,) = struct.unpack("=l", raw[pos:pos + 4])
        bodies.append(raw[pos + 4:pos + 4 + n])
        pos += 4 + n
    assert sorted(bodies) == sorted(written)
    for b_ in bodies:
        ep = msgs["Episode"]()
        ep.ParseFromString(b_)
        assert len(ep.event[0].action) == 0


def test_writer_errors():
    lib = native.load()
    h = C.c_void_p()
    assert lib.cp_eventlog_open(b"/nonexistent-dir/x.log", 2, C.byref(h)) != 0
    assert b"cannot open" in lib.cp_last_error(None)
    assert lib.cp_event_record_bytes(7, 3, 1) < 0
