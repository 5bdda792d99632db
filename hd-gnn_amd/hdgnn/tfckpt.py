"""TensorFlow V2 checkpoint (tensor bundle) reader / writer, numpy only.

The reference saves with tf.train.Saver (model_2.py:139, 427-437) and restores through
tf.train.get_checkpoint_state + saver.restore (439-451).  A V2 checkpoint "<prefix>" is

    <prefix>.index                  an SSTable (LevelDB table format): key "" -> the bundle
                                    header proto, key <variable name> -> its entry proto
    <prefix>.data-00000-of-00001    the tensors' raw little-endian bytes, back to back
    checkpoint                      text proto naming the latest prefix

Formats restated from their public definitions (TensorFlow tensor_bundle.proto /
tensor_shape.proto / versions.proto, LevelDB doc/table_format.md, the Snappy framing-free
format):
    SSTable block   entries (varint shared, varint non_shared, varint value_len, key delta,
                    value) + uint32 restart offsets + uint32 restart count; each block on
                    disk is followed by a 1-byte compression type (0 none, 1 snappy) and the
                    masked CRC-32C of contents + type byte
    footer (48 B)   metaindex handle, index handle (varint64 offset, size each), zero pad
                    to 40 B, fixed64 magic 0xdb4775248b80fb57
    header proto    num_shards=1 (int32), endianness=2 (enum, 0 little), version=3
                    (VersionDef: producer=1, min_consumer=2)
    entry proto     dtype=1 (enum), shape=2 (TensorShapeProto: dim=2 {size=1}), shard_id=3,
                    offset=4, size=5, crc32c=6 (fixed32, masked CRC-32C of the bytes),
                    slices=7 (partitioned variables: not supported, raises)
    mask(crc)       ((crc >> 15) | (crc << 17)) + 0xa282ead8  (mod 2^32)

The reference's Saver is built before its AdamOptimizer (model_2.py:139 vs 337), so its
checkpoints hold the model variables only; write() can add TF1 Adam's slot names
(<var>/Adam, <var>/Adam_1, beta1_power, beta2_power), which a TF Saver that has them
restores and one that does not ignores.

Parity: no TF-written checkpoint exists in the reference snapshot and TensorFlow is not
installed, so reading real TF files is "parity unpinned"; tests/test_tfckpt.py pins the
container format by hand-built SSTables, CRC-32C / Snappy known answers and round trips.
"""
import os
import functools
import struct

import numpy as np

MAGIC = 0xdb4775248b80fb57
_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8,
           9: np.int64, 10: np.bool_, 17: np.uint16, 22: np.uint32, 23: np.uint64}
_DT_OF = {np.dtype(v).str: k for k, v in _DTYPES.items()}


class CheckpointError(ValueError):
    pass


# ------------------------------------------------------------------ CRC-32C (Castagnoli)
def _crc_table():
    poly = 0x82F63B78
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        t.append(c)
    return t


_CRC_T = _crc_table()


def crc32c_py(data, crc=0):
    c = crc ^ 0xFFFFFFFF
    t = _CRC_T
    for b in bytes(data):
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _crc_impl():
    """libhdgnn's slicing-by-8 CRC-32C when the library is built (a bundle write is
    checksum-bound in Python: ~5 ms per model_2 checkpoint), else the table loop above."""
    try:
        from . import _lib
        lib = _lib.load()
        return lambda data, crc=0: int(lib.hdg_crc32c(bytes(data), len(data), crc))
    except Exception:
        return crc32c_py


_CRC_FN = None


def crc32c(data, crc=0):
    global _CRC_FN
    if _CRC_FN is None:
        _CRC_FN = _crc_impl()
    return _CRC_FN(data, crc)


def mask_crc(c):
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xa282ead8) & 0xFFFFFFFF


# ------------------------------------------------------------------ varints / protobuf
_VARINT1 = [bytes((i,)) for i in range(128)]   # one-byte varints (most of a bundle's)


def _put_varint(v):
    if 0 <= v < 128:
        return _VARINT1[v]
    if v < 0:
        v &= (1 << 64) - 1           # protobuf int32/int64: negatives as 10-byte varints
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _get_varint(buf, pos):
    v = shift = 0
    while True:
        if pos >= len(buf):
            raise CheckpointError("truncated varint")
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, pos
        shift += 7
        if shift > 63:
            raise CheckpointError("varint too long")


def _pb_fields(buf):
    """Decode one protobuf message -> list of (field, wire_type, value)."""
    out, pos = [], 0
    while pos < len(buf):
        tag, pos = _get_varint(buf, pos)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, pos = _get_varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _get_varint(buf, pos)
            v = bytes(buf[pos:pos + n])
            if len(v) != n:
                raise CheckpointError("truncated length-delimited field")
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise CheckpointError("unsupported wire type %d" % wt)
        out.append((f, wt, v))
    return out


def _pb_varint(f, v):
    return _put_varint(f << 3) + _put_varint(v)


def _pb_bytes(f, b):
    return _put_varint((f << 3) | 2) + _put_varint(len(b)) + b


def _pb_fixed32(f, v):
    return _put_varint((f << 3) | 5) + struct.pack("<I", v)


def _signed64(v):
    return v - (1 << 64) if v >= 1 << 63 else v


def encode_header(num_shards=1):
    version = _pb_varint(1, 1)                      # producer = kTensorBundleVersion
    return _pb_varint(1, num_shards) + _pb_bytes(3, version)   # endianness LITTLE = default


@functools.lru_cache(maxsize=4096)
def _entry_head(dtype_enum, shape, shard_id, offset, size):
    """BundleEntryProto fields 1-5 (a checkpoint of fixed shapes repeats them every save)."""
    shp = b"".join(_pb_bytes(2, _pb_varint(1, int(d))) for d in shape)
    msg = _pb_varint(1, dtype_enum) + _pb_bytes(2, shp)
    if shard_id:
        msg += _pb_varint(3, shard_id)
    if offset:
        msg += _pb_varint(4, offset)
    return msg + _pb_varint(5, size)


def encode_entry(dtype_enum, shape, shard_id, offset, size, masked_crc):
    return (_entry_head(int(dtype_enum), tuple(int(d) for d in shape), int(shard_id),
                        int(offset), int(size)) + _pb_fixed32(6, masked_crc))


def decode_entry(buf):
    e = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": None,
         "slices": 0}
    for f, wt, v in _pb_fields(buf):
        if f == 1 and wt == 0:
            e["dtype"] = v
        elif f == 2 and wt == 2:
            for g, gwt, gv in _pb_fields(v):
                if g == 2 and gwt == 2:
                    size = -1
                    for h, hwt, hv in _pb_fields(gv):
                        if h == 1 and hwt == 0:
                            size = _signed64(hv)
                    e["shape"].append(size)
                elif g == 3 and gwt == 0 and gv:
                    raise CheckpointError("unknown-rank tensor in checkpoint")
        elif f == 3 and wt == 0:
            e["shard_id"] = v
        elif f == 4 and wt == 0:
            e["offset"] = _signed64(v)
        elif f == 5 and wt == 0:
            e["size"] = _signed64(v)
        elif f == 6 and wt == 5:
            e["crc32c"] = v
        elif f == 7:
            e["slices"] += 1
    return e


def decode_header(buf):
    h = {"num_shards": 0, "endianness": 0, "producer": 0, "min_consumer": 0}
    for f, wt, v in _pb_fields(buf):
        if f == 1 and wt == 0:
            h["num_shards"] = v
        elif f == 2 and wt == 0:
            h["endianness"] = v
        elif f == 3 and wt == 2:
            for g, gwt, gv in _pb_fields(v):
                if g == 1 and gwt == 0:
                    h["producer"] = gv
                elif g == 2 and gwt == 0:
                    h["min_consumer"] = gv
    return h


# ------------------------------------------------------------------ Snappy (raw format)
def snappy_decompress(buf):
    n, pos = _get_varint(buf, 0)
    out = bytearray()
    while pos < len(buf):
        tag = buf[pos]
        pos += 1
        kind = tag & 3
        if kind == 0:                                 # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(buf[pos:pos + nb], "little")
                pos += nb
            ln += 1
            if pos + ln > len(buf):
                raise CheckpointError("snappy literal overruns the block")
            out += buf[pos:pos + ln]
            pos += ln
            continue
        if kind == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | buf[pos]
            pos += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[pos:pos + 2], "little")
            pos += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[pos:pos + 4], "little")
            pos += 4
        if off == 0 or off > len(out):
            raise CheckpointError("snappy copy offset out of range")
        for _ in range(ln):                           # overlapping copies are legal
            out.append(out[-off])
    if len(out) != n:
        raise CheckpointError("snappy length mismatch (%d != %d)" % (len(out), n))
    return bytes(out)


# ------------------------------------------------------------------ SSTable
def _read_block(data, offset, size, verify=True):
    if offset + size + 5 > len(data):
        raise CheckpointError("block handle beyond end of index file")
    contents = data[offset:offset + size]
    ctype = data[offset + size]
    if verify:
        want = struct.unpack_from("<I", data, offset + size + 1)[0]
        if mask_crc(crc32c(data[offset:offset + size + 1])) != want:
            raise CheckpointError("index block checksum mismatch at offset %d" % offset)
    if ctype == 0:
        return contents
    if ctype == 1:
        return snappy_decompress(contents)
    raise CheckpointError("unknown block compression type %d" % ctype)


def _block_entries(block):
    if len(block) < 4:
        raise CheckpointError("block too short")
    nres = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * nres
    if end < 0:
        raise CheckpointError("bad restart count")
    pos, key = 0, b""
    while pos < end:
        shared, pos = _get_varint(block, pos)
        nshared, pos = _get_varint(block, pos)
        vlen, pos = _get_varint(block, pos)
        if shared > len(key):
            raise CheckpointError("bad key prefix length")
        key = key[:shared] + bytes(block[pos:pos + nshared])
        pos += nshared
        val = bytes(block[pos:pos + vlen])
        pos += vlen
        yield key, val


def read_table(data, verify=True):
    """All (key, value) pairs of an SSTable image, in file order."""
    if len(data) < 48:
        raise CheckpointError("index file shorter than the table footer")
    foot = data[-48:]
    if struct.unpack_from("<Q", foot, 40)[0] != MAGIC:
        raise CheckpointError("not an SSTable (bad magic)")
    _, p = _get_varint(foot, 0)
    _, p = _get_varint(foot, p)                       # metaindex handle (unused)
    ioff, p = _get_varint(foot, p)
    isz, p = _get_varint(foot, p)
    out = []
    for _, hv in _block_entries(_read_block(data, ioff, isz, verify)):
        boff, q = _get_varint(hv, 0)
        bsz, _ = _get_varint(hv, q)
        out.extend(_block_entries(_read_block(data, boff, bsz, verify)))
    return out


def _block_bytes(entries, restart_interval=16, vpos=None):
    """One block's contents; vpos (a list) receives each entry's value offset in it."""
    buf, restarts, prev = bytearray(), [], b""
    for n, (k, v) in enumerate(entries):
        if n % restart_interval == 0:
            restarts.append(len(buf))
            shared = 0
        else:
            shared = 0
            m = min(len(prev), len(k))
            while shared < m and prev[shared] == k[shared]:
                shared += 1
        buf += _put_varint(shared) + _put_varint(len(k) - shared) + _put_varint(len(v))
        buf += k[shared:]
        if vpos is not None:
            vpos.append(len(buf))
        buf += v
        prev = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        buf += struct.pack("<I", r)
    buf += struct.pack("<I", len(restarts))
    return bytes(buf)


def write_table(entries, block_size=4096, layout=None):
    """Sorted (key, value) pairs -> SSTable image (uncompressed blocks, no filter).
    layout (a dict) receives "values": each entry's absolute value offset in the image and
    "blocks": (offset, length) of every block, in the order their checksums depend on."""
    keys = [k for k, _ in entries]
    if keys != sorted(keys) or len(set(keys)) != len(keys):
        raise CheckpointError("table keys must be unique and sorted")
    out = bytearray()
    index = []
    values, blocks = [], []

    def emit(contents, vpos=None):
        off = len(out)
        out.extend(contents)
        tail = b"\x00"
        out.extend(tail + struct.pack("<I", mask_crc(crc32c(contents + tail))))
        values.extend(off + p for p in (vpos or ()))
        blocks.append((off, len(contents)))
        return _put_varint(off) + _put_varint(len(contents))

    def data_block(cur):
        vpos = []
        return emit(_block_bytes(cur, vpos=vpos), vpos)

    cur, size = [], 0
    for k, v in entries:
        cur.append((k, v))
        size += len(k) + len(v) + 8
        if size >= block_size:
            index.append((cur[-1][0], data_block(cur)))
            cur, size = [], 0
    if cur:
        index.append((cur[-1][0], data_block(cur)))
    meta = emit(_block_bytes([]))
    idx = emit(_block_bytes(index, restart_interval=1))
    foot = meta + idx
    foot += b"\x00" * (40 - len(foot)) + struct.pack("<Q", MAGIC)
    out.extend(foot)
    if layout is not None:
        layout["values"], layout["blocks"] = values, blocks
    return bytes(out)


# ------------------------------------------------------------------ bundles
def _shard_name(prefix, i, n):
    return "%s.data-%05d-of-%05d" % (prefix, i, n)


def read(prefix, verify=True):
    """<prefix>.index + data shards -> {variable name: ndarray} (TF names, no ':0')."""
    with open(prefix + ".index", "rb") as f:
        data = f.read()
    entries = read_table(data, verify)
    if not entries or entries[0][0] != b"":
        raise CheckpointError("bundle header entry missing")
    hdr = decode_header(entries[0][1])
    if hdr["endianness"] != 0:
        raise CheckpointError("big-endian bundles are not supported")
    nsh = max(hdr["num_shards"], 1)
    shards = {}
    out = {}
    for key, val in entries[1:]:
        e = decode_entry(val)
        name = key.decode("utf-8")
        if e["slices"]:
            raise CheckpointError("%s is a partitioned (sliced) variable" % name)
        if e["dtype"] not in _DTYPES:
            raise CheckpointError("%s: unsupported dtype enum %d" % (name, e["dtype"]))
        sid = e["shard_id"]
        if sid not in shards:
            with open(_shard_name(prefix, sid, nsh), "rb") as f:
                shards[sid] = f.read()
        raw = shards[sid][e["offset"]:e["offset"] + e["size"]]
        if len(raw) != e["size"]:
            raise CheckpointError("%s: data shard too short" % name)
        if verify and e["crc32c"] is not None and mask_crc(crc32c(raw)) != e["crc32c"]:
            raise CheckpointError("%s: tensor checksum mismatch" % name)
        dt = np.dtype(_DTYPES[e["dtype"]]).newbyteorder("<")
        shape = tuple(e["shape"])
        arr = np.frombuffer(raw, dtype=dt)
        if arr.size != int(np.prod(shape, dtype=np.int64)):
            raise CheckpointError("%s: %d elements for shape %s" % (name, arr.size, shape))
        out[name] = arr.reshape(shape).astype(dt.newbyteorder("="), copy=True)
    return out


def write(prefix, tensors):
    """{name: ndarray} -> <prefix>.index + <prefix>.data-00000-of-00001 (one shard, keys
    in byte order as TF's BundleWriter requires)."""
    names = sorted(tensors, key=lambda n: n.encode("utf-8"))
    blob = bytearray()
    entries = [(b"", encode_header(1))]
    for n in names:
        a = np.asarray(tensors[n])           # (ascontiguousarray would make 0-d 1-d)
        dt = a.dtype.newbyteorder("<")
        if dt.str not in _DT_OF:
            raise CheckpointError("%s: dtype %s has no TF enum here" % (n, a.dtype))
        raw = a.astype(dt, copy=False).tobytes()
        entries.append((n.encode("utf-8"),
                        encode_entry(_DT_OF[dt.str], a.shape, 0, len(blob), len(raw),
                                     mask_crc(crc32c(raw)))))
        blob += raw
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(_shard_name(prefix, 0, 1), "wb") as f:
        f.write(bytes(blob))
    with open(prefix + ".index", "wb") as f:
        f.write(write_table(entries))


class BundleTemplate(object):
    """The byte layout of one model variant's training checkpoint (model variables, TF1 Adam
    slots, beta powers: every tensor float32, fixed shapes), built once.  write() fills it
    from the flat engine state [params | adam_m | adam_v | beta_pow] (Engine.state, slices at
    layout.state_offsets) in libhdgnn's
    hdg_bundle_write: the tensor bytes gathered in name order, each entry's CRC and each
    index block's trailer CRC patched into the index image, both files written -- native
    code that runs with the GIL released (ctypes), so the saver thread does not stall the
    training loop.  Same bytes as write(prefix, state_tensors(...)) (tests/test_tfckpt.py)."""

    def __init__(self, variant, slots=True):
        from . import layout
        sl = _var_slices(variant)
        P = sum(n for _, _, n, _ in sl)
        so = layout.state_offsets(variant)
        spans = {}
        for base, o, n, shape in sl:
            spans[base] = (o, n, shape)
            if slots:
                spans[base + "/Adam"] = (so["m"] + o, n, shape)
                spans[base + "/Adam_1"] = (so["v"] + o, n, shape)
        if slots:
            spans["beta1_power"] = (so["beta_pow"], 1, ())
            spans["beta2_power"] = (so["beta_pow"] + 1, 1, ())
        self.n_state = so["len"] if slots else P
        names = sorted(spans, key=lambda n: n.encode("utf-8"))
        gather, entries, offs = [], [(b"", encode_header(1))], []
        nbytes = 0
        for n in names:
            o, cnt, shape = spans[n]
            gather.extend(range(o, o + cnt))
            entries.append((n.encode("utf-8"), encode_entry(1, shape, 0, nbytes, 4 * cnt, 0)))
            offs.append((nbytes, 4 * cnt))
            nbytes += 4 * cnt
        lay = {}
        img = write_table(entries, layout=lay)
        # entry e's CRC is the last 4 bytes of its value (entry proto field 6, fixed32)
        ent = [(off, size, vp + len(entries[i + 1][1]) - 4)
               for i, ((off, size), vp) in enumerate(zip(offs, lay["values"][1:]))]
        self.gather = np.asarray(gather, np.int32)
        self.entries = np.asarray(ent, np.int64).reshape(-1, 3)
        self.blocks = np.asarray(lay["blocks"], np.int64).reshape(-1, 2)
        self.image = np.frombuffer(img, np.uint8).copy()

    def write(self, prefix, state):
        from . import _lib
        state = np.ascontiguousarray(state, np.float32)
        if state.size != self.n_state:
            raise CheckpointError("state has %d floats, the template %d" % (state.size, self.n_state))
        d = os.path.dirname(prefix)
        if d:
            os.makedirs(d, exist_ok=True)
        img = self.image.copy()
        lib = _lib.load()
        _lib.check(lib.hdg_bundle_write(
            _shard_name(prefix, 0, 1).encode(), (prefix + ".index").encode(),
            state.ctypes.data, state.size, self.gather.ctypes.data, self.gather.size,
            img.ctypes.data,
            img.size, self.entries.ctypes.data, len(self.entries), self.blocks.ctypes.data,
            len(self.blocks)))


class BundleWriter(object):
    """libhdgnn's background writer (hdg_ckpt_writer_*) over a BundleTemplate: one native
    thread writes the queued bundles and text files in submission order, so the training
    loop's thread only hands over a copy of the state (no Python runs on the writer, nothing
    holds the GIL while it writes).  flush() waits for the queue and raises the first
    failure since the previous flush."""

    def __init__(self, template):
        import ctypes
        from . import _lib
        self._lib = _lib.load()
        self._t = template
        h = ctypes.c_void_p()
        _lib.check(self._lib.hdg_ckpt_writer_create(
            template.gather.ctypes.data, template.gather.size, template.n_state,
            template.image.ctypes.data, template.image.size, template.entries.ctypes.data,
            len(template.entries), template.blocks.ctypes.data, len(template.blocks),
            ctypes.byref(h)))
        self._h = h

    @staticmethod
    def _b(v):
        return None if v is None else v.encode("utf-8")

    def submit(self, prefix=None, state=None, removes=(), text_path=None, text=None,
               append=False):
        """Queue: the bundle of `state` at `prefix` (if given), then delete `removes`, then
        write (or append) `text` to `text_path` (if given)."""
        if state is not None:
            state = np.ascontiguousarray(state, np.float32)
            if state.size != self._t.n_state:
                raise CheckpointError("state has %d floats, the template %d"
                                      % (state.size, self._t.n_state))
        rm = "\n".join(removes) if removes else None
        rc = self._lib.hdg_ckpt_writer_submit(
            self._h, None if state is None else state.ctypes.data,
            self._b(None if prefix is None else _shard_name(prefix, 0, 1)),
            self._b(None if prefix is None else prefix + ".index"), self._b(rm),
            self._b(text_path), self._b(text), 1 if append else 0)
        if rc:
            raise CheckpointError(self._lib.hdg_last_error().decode(errors="replace"))

    def flush(self):
        if self._h is not None and self._lib.hdg_ckpt_writer_flush(self._h):
            raise CheckpointError(self._lib.hdg_last_error().decode(errors="replace"))

    def poll(self):
        """Raise the first failure since the last flush / poll, without waiting."""
        if self._h is not None and self._lib.hdg_ckpt_writer_poll(self._h):
            raise CheckpointError(self._lib.hdg_last_error().decode(errors="replace"))

    def close(self):
        h, self._h = self._h, None
        if h is not None and self._lib.hdg_ckpt_writer_destroy(h):
            raise CheckpointError(self._lib.hdg_last_error().decode(errors="replace"))

    def __del__(self):
        import sys
        if not sys.is_finalizing():
            try:
                self.close()
            except Exception:
                pass


def latest(checkpoint_dir):
    """tf.train.get_checkpoint_state(dir).model_checkpoint_path's basename, or None."""
    p = os.path.join(checkpoint_dir, "checkpoint")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        for line in f:
            line = line.strip()
            if line.startswith("model_checkpoint_path:"):
                v = line.split(":", 1)[1].strip()
                if len(v) >= 2 and v[0] == v[-1] == '"':
                    v = v[1:-1].encode("latin-1").decode("unicode_escape")
                return os.path.basename(v)
    return None


def state_file_text(name, all_names=None):
    """The CheckpointState text proto tf.train.Saver.save writes next to the bundles:
    the latest prefix and every prefix still kept (max_to_keep), oldest first."""
    return ('model_checkpoint_path: "%s"\n' % name +
            "".join('all_model_checkpoint_paths: "%s"\n' % n for n in (all_names or [name])))


def write_state_file(checkpoint_dir, name, all_names=None):
    with open(os.path.join(checkpoint_dir, "checkpoint"), "w") as f:
        f.write(state_file_text(name, all_names))


def remove_bundle(prefix):
    """Delete the files of the bundle at prefix (index + data shards), as Saver does for
    checkpoints that fall out of max_to_keep."""
    d, base = os.path.split(prefix)
    for f in os.listdir(d or "."):
        if f == base + ".index" or f.startswith(base + ".data-"):
            os.remove(os.path.join(d, f))


# ------------------------------------------------------------------ engine state <-> TF names
@functools.lru_cache(maxsize=None)
def _var_slices(variant):
    """(TF name without ':0', offset, size, shape) of every variable of the flat vector."""
    from . import layout
    return tuple((name.split(":")[0], o, int(np.prod(shape)), tuple(shape))
                 for name, (o, shape) in layout.offsets(variant).items())


def state_tensors(flat, variant, adam_m=None, adam_v=None, beta_pow=None):
    """Flat engine vectors -> TF-named tensors (model variables, optional TF1 Adam slots)."""
    flat = np.asarray(flat, np.float32)
    if adam_m is not None:
        adam_m, adam_v = np.asarray(adam_m, np.float32), np.asarray(adam_v, np.float32)
    out = {}
    for base, o, n, shape in _var_slices(variant):
        out[base] = flat[o:o + n].reshape(shape)
        if adam_m is not None:
            out[base + "/Adam"] = adam_m[o:o + n].reshape(shape)
            out[base + "/Adam_1"] = adam_v[o:o + n].reshape(shape)
    if beta_pow is not None:
        out["beta1_power"] = np.asarray(beta_pow[0], np.float32).reshape(())
        out["beta2_power"] = np.asarray(beta_pow[1], np.float32).reshape(())
    return out


def engine_state(tensors, variant):
    """TF-named tensors -> (flat, adam_m | None, adam_v | None, beta_pow | None); every model
    variable must be present with its shape (what saver.restore requires)."""
    from . import layout
    parts, ms, vs = [], [], []
    have_slots = True
    for name, shape in layout.specs(variant):
        base = name.split(":")[0]
        if base not in tensors:
            raise CheckpointError("checkpoint lacks variable %s (model_%d)" % (base, variant))
        a = np.asarray(tensors[base])
        if tuple(a.shape) != tuple(shape):
            raise CheckpointError("%s: shape %s in checkpoint, %s in model_%d"
                                  % (base, a.shape, shape, variant))
        parts.append(a.astype(np.float32).reshape(-1))
        if base + "/Adam" in tensors and base + "/Adam_1" in tensors:
            ms.append(np.asarray(tensors[base + "/Adam"], np.float32).reshape(-1))
            vs.append(np.asarray(tensors[base + "/Adam_1"], np.float32).reshape(-1))
        else:
            have_slots = False
    flat = np.concatenate(parts)
    if have_slots and "beta1_power" in tensors and "beta2_power" in tensors:
        bp = np.array([float(tensors["beta1_power"]), float(tensors["beta2_power"])], np.float32)
        return flat, np.concatenate(ms), np.concatenate(vs), bp
    return flat, None, None, None
