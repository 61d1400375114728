"""Event log: episodes of (action, state, reward) events in the reference's protobuf
wire format (event.proto:1-35) with its '=l' length-prefix framing
(event_log.py:48-58 writer, :103-111 reader), so `ReplayMemory.reset_from_event_log`
(replay_memory.py:40-61) can ingest rollouts of the MI355X env.

Two writers produce the same bytes:
  - `EventLog` (single env; the reference's class API: reset / add / add_just_state),
    encoding in Python, pixel states as PNG renders like the reference;
  - `BatchedEventLog` (B envs on the GPU): the step's events are encoded by a HIP kernel
    (`cp_encode_events`, one fixed-size record per env) and appended to per-env episode
    buffers by the native host writer (`cp_eventlog_*`), which frames and writes an
    episode when its env is reset.
`EventLogReader` / `read_state_from_event` read both (and the reference's logs).

Wire format (proto2: repeated scalars are not packed, fields in number order):
  Episode { repeated Event event = 1; }
  Event   { repeated float action = 1; repeated State state = 2; optional float reward = 3; }
  State   { repeated float cart_pose = 1; repeated float pole_pose = 2; repeated Render render = 3; }
  Render  { optional int32 height = 1; optional int32 width = 2; optional bytes png_bytes = 3; }
"""
import ctypes as C
import gzip
import struct
import zlib

import numpy as np

# ----------------------------------------------------------------- encoding


def _varint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field, wire):
    return _varint((field << 3) | wire)


def _f32(field, x):
    return _key(field, 5) + struct.pack("<f", float(x))


def _ld(field, payload):
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_render(height, width, png_bytes):
    return _key(1, 0) + _varint(int(height)) + _key(2, 0) + _varint(int(width)) + _ld(3, png_bytes)


def encode_state_lowdim(cart_pose, pole_pose):
    """State with the 7d cart and pole poses (event.proto:10-15)."""
    return b"".join(_f32(1, x) for x in cart_pose) + b"".join(_f32(2, x) for x in pole_pose)


def encode_state_renders(renders):
    """State with one Render per camera: renders = [(height, width, png_bytes), ...]."""
    return b"".join(_ld(3, encode_render(*r)) for r in renders)


def encode_event(states, action=None, reward=None):
    """Event bytes from encoded States (event.proto:23-30)."""
    out = b""
    if action is not None:
        out += b"".join(_f32(1, a) for a in action)
    out += b"".join(_ld(2, s) for s in states)
    if reward is not None:
        out += _f32(3, reward)
    return out


def episode_entry(event_bytes):
    """One `event` field of an Episode (the unit the batched writer appends)."""
    return _ld(1, event_bytes)


# ---------------------------------------------------------------------- PNG


def rgb_to_png(rgb):
    """RGB in [0, 1] (H, W, 3) -> 8-bit RGB PNG (the reference uses plt.imsave, :8-12)."""
    a = np.clip(np.asarray(rgb, dtype=np.float64), 0.0, 1.0)
    u8 = np.floor(a * 255.0 + 0.5).astype(np.uint8)
    h, w, _ = u8.shape
    raw = b"".join(b"\x00" + u8[y].tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) +
            chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b""))


def png_to_rgb(png_bytes):
    """8-bit RGB / RGBA PNG (filter type 0 rows, as rgb_to_png writes) -> float32 RGB in
    [0, 1] (the reference's png_to_rgb slices RGBA to RGB, :14-18)."""
    assert png_bytes[:8] == b"\x89PNG\r\n\x1a\n", "not a PNG"
    pos, idat = 8, b""
    w = h = ch = None
    while pos < len(png_bytes):
        (n,) = struct.unpack(">I", png_bytes[pos:pos + 4])
        t = png_bytes[pos + 4:pos + 8]
        d = png_bytes[pos + 8:pos + 8 + n]
        if t == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", d[:10])
            assert depth == 8 and ctype in (2, 6), "only 8-bit RGB/RGBA PNGs"
            ch = 3 if ctype == 2 else 4
        elif t == b"IDAT":
            idat += d
        pos += 12 + n
    raw = zlib.decompress(idat)
    stride = w * ch + 1
    rows = [raw[y * stride:(y + 1) * stride] for y in range(h)]
    assert all(r[0] == 0 for r in rows), "only unfiltered rows"
    img = np.frombuffer(b"".join(r[1:] for r in rows), np.uint8).reshape(h, w, ch)
    return img[:, :, :3].astype(np.float32) / 255.0


# ----------------------------------------------------------------- decoding


class Render:
    def __init__(self):
        self.height = 0
        self.width = 0
        self.png_bytes = b""


class State:
    def __init__(self):
        self.cart_pose = []
        self.pole_pose = []
        self.render = []


class Event:
    def __init__(self):
        self.action = []
        self.state = []
        self.reward = 0.0
        self._has_reward = False

    def HasField(self, name):  # noqa: N802 - protobuf message API
        assert name == "reward", name
        return self._has_reward


class Episode:
    def __init__(self):
        self.event = []


def _fields(buf):
    """Yield (field, wire, value) of a protobuf message."""
    pos = 0
    n = len(buf)
    while pos < n:
        key, pos = _read_varint(buf, pos)
        field, wire = key >> 3, key & 7
        if wire == 0:
            v, pos = _read_varint(buf, pos)
        elif wire == 5:
            v = struct.unpack_from("<f", buf, pos)[0]
            pos += 4
        elif wire == 2:
            ln, pos = _read_varint(buf, pos)
            v = buf[pos:pos + ln]
            pos += ln
        elif wire == 1:
            v = struct.unpack_from("<d", buf, pos)[0]
            pos += 8
        else:
            raise ValueError(f"unsupported wire type {wire}")
        yield field, wire, v


def _read_varint(buf, pos):
    shift = result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _floats(wire, v):
    if wire == 5:
        return [v]
    return list(struct.unpack(f"<{len(v) // 4}f", v))  # packed (a writer may pack)


def parse_render(buf):
    r = Render()
    for f, w, v in _fields(buf):
        if f == 1:
            r.height = v
        elif f == 2:
            r.width = v
        elif f == 3:
            r.png_bytes = bytes(v)
    return r


def parse_state(buf):
    s = State()
    for f, w, v in _fields(buf):
        if f == 1:
            s.cart_pose += _floats(w, v)
        elif f == 2:
            s.pole_pose += _floats(w, v)
        elif f == 3:
            s.render.append(parse_render(v))
    return s


def parse_event(buf):
    e = Event()
    for f, w, v in _fields(buf):
        if f == 1:
            e.action += _floats(w, v)
        elif f == 2:
            e.state.append(parse_state(v))
        elif f == 3:
            e.reward = v
            e._has_reward = True
    return e


def parse_episode(buf):
    ep = Episode()
    for f, w, v in _fields(buf):
        if f == 1:
            ep.event.append(parse_event(v))
    return ep


def read_state_from_event(event):
    """Inverse of add_state_to_event (event_log.py:21-39): (H, W, 3, C, R) renders or
    (R, 2, 7) poses."""
    if len(event.state[0].render) > 0:
        num_repeats = len(event.state)
        num_cameras = len(event.state[0].render)
        eg = event.state[0].render[0]
        state = np.empty((eg.height, eg.width, 3, num_cameras, num_repeats))
        for r_idx in range(num_repeats):
            for c_idx in range(num_cameras):
                state[:, :, :, c_idx, r_idx] = png_to_rgb(event.state[r_idx].render[c_idx].png_bytes)
    else:
        state = np.empty((len(event.state), 2, 7))
        for i, s in enumerate(event.state):
            state[i][0] = s.cart_pose
            state[i][1] = s.pole_pose
    return state


class EventLogReader:
    """event_log.py:101-118: '=l'-prefixed Episode messages, optionally gzipped."""

    def __init__(self, path):
        self.log_file = gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")

    def entries(self):
        while True:
            n = self.log_file.read(4)
            if len(n) == 0:
                return
            (ln,) = struct.unpack("=l", n)
            yield parse_episode(self.log_file.read(ln))


# ------------------------------------------------------------------ writers


class EventLog:
    """Single-env writer with the reference's API (event_log.py:42-99)."""

    def __init__(self, path, use_raw_pixels):
        self.log_file = open(path, "ab")
        self.episode = None           # encoded Episode so far (bytes)
        self.use_raw_pixels = use_raw_pixels

    def reset(self):
        if self.episode:
            self.log_file.write(struct.pack("=l", len(self.episode)))
            self.log_file.write(self.episode)
            self.log_file.flush()
        self.episode = b""

    def _states(self, state):
        if self.use_raw_pixels:       # (H, W, 3, C, R)
            return [encode_state_renders([(state.shape[0], state.shape[1], rgb_to_png(state[:, :, :, c, r]))
                                          for c in range(state.shape[3])]) for r in range(state.shape[4])]
        return [encode_state_lowdim(state[r][0], state[r][1]) for r in range(state.shape[0])]

    def add(self, state, action, reward):
        if isinstance(action, (int, np.integer)):
            act = [action]
        else:
            act = [float(a) for a in np.asarray(action, dtype=np.float64).reshape(-1)]
        self.episode += episode_entry(encode_event(self._states(state), act, reward))

    def add_just_state(self, state):
        self.episode += episode_entry(encode_event(self._states(state)))

    def close(self):
        self.reset()
        self.log_file.close()


class BatchedEventLog:
    """Event log of a BatchedCartpole (low-dim obs): GPU-encoded records, native writer.

        log = BatchedEventLog(env, "rollouts.log")
        obs = env.reset();          log.after_reset()
        obs, r, d = env.step(a);    log.after_step(a)
        log.close()
    Each env's episode (its reset event, then one event per simulated step) is framed and
    written when that env is reset again (autoreset: in the same step), and at close()."""

    def __init__(self, env, path):
        import torch
        from . import native
        self.env, self.lib = env, native.load()
        self.h = C.c_void_p()
        native.check(None, self.lib.cp_eventlog_open(path.encode(), env.B, C.byref(self.h)), "cp_eventlog_open")
        self._torch, self._native = torch, native
        dev = env.device
        self.flags = torch.zeros(env.B, dtype=torch.uint8, device=dev)
        self._bufs = {}

    def _records(self, kind):
        if kind not in self._bufs:
            sb = self.lib.cp_event_record_bytes(kind, self.env.R, 1)
            rb = self.lib.cp_event_record_bytes(kind, self.env.R, 0)
            t = self._torch
            self._bufs[kind] = (sb, rb, t.zeros((self.env.B, sb), dtype=t.uint8, device=self.env.device),
                                t.zeros((self.env.B, rb), dtype=t.uint8, device=self.env.device))
        return self._bufs[kind]

    def _write(self, kind):
        sb, rb, step_rec, reset_rec = self._records(kind)
        f = self.flags.cpu().numpy()
        s = step_rec.cpu().numpy()
        r = reset_rec.cpu().numpy()
        self._native.check(self.h, self.lib.cp_eventlog_write(self.h, f.ctypes.data, s.ctypes.data, sb,
                                                              r.ctypes.data, rb), "cp_eventlog_write")

    def after_reset(self, mask=None, kind=None):
        from . import abi
        kind = abi.CP_ACTION_DISCRETE if (kind is None and self.env.discrete_actions) else (
            abi.CP_ACTION_CONTINUOUS if kind is None else kind)
        sb, rb, step_rec, reset_rec = self._records(kind)
        m = None if mask is None else self._torch.as_tensor(mask, device=self.env.device).to(self._torch.uint8)
        e = self.env
        self._native.check(e.h, self.lib.cp_encode_events(
            e.h, 1, None, kind, C.c_void_p(e.obs.data_ptr()), None, None, None,
            None if m is None else C.c_void_p(m.data_ptr()), C.c_void_p(step_rec.data_ptr()),
            C.c_void_p(reset_rec.data_ptr()), C.c_void_p(self.flags.data_ptr()), e._stream()), "cp_encode_events")
        self._write(kind)

    def after_step(self, actions):
        from . import abi
        t = self._torch
        kind = abi.CP_ACTION_DISCRETE if actions.dtype == t.int8 else abi.CP_ACTION_CONTINUOUS
        actions = actions.to(self.env.device).contiguous()
        if kind == abi.CP_ACTION_CONTINUOUS:
            actions = actions.float()
        sb, rb, step_rec, reset_rec = self._records(kind)
        e = self.env
        term = e.terminal_obs
        self._native.check(e.h, self.lib.cp_encode_events(
            e.h, 0, C.c_void_p(actions.data_ptr()), kind, C.c_void_p(e.obs.data_ptr()),
            None if term is None else C.c_void_p(term.data_ptr()), C.c_void_p(e.reward.data_ptr()),
            C.c_void_p(e.done.data_ptr()), None, C.c_void_p(step_rec.data_ptr()), C.c_void_p(reset_rec.data_ptr()),
            C.c_void_p(self.flags.data_ptr()), e._stream()), "cp_encode_events")
        self._write(kind)

    def close(self):
        if self.h:
            self.lib.cp_eventlog_close(self.h)
            self.h = None
