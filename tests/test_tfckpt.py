"""TF V2 checkpoint reader / writer (hdgnn.tfckpt).  CPU only.

Parity against TF-written files is unpinned (no TensorFlow here and no checkpoint in the
reference snapshot); the container format is pinned piece by piece: CRC-32C known answers
(RFC 3720 B.4), a Snappy stream and an SSTable assembled by hand from the published
formats, then round trips and corruption detection.
"""
import os
import struct

import numpy as np
import pytest

from hdgnn import layout, tfckpt


@pytest.mark.parametrize("data,want", [
    (b"123456789", 0xE3069283),
    (bytes(32), 0x8A9136AA),
    (b"\xff" * 32, 0x62A8AB43),
    (bytes(range(32)), 0x46DD794E),
    (bytes(range(31, -1, -1)), 0x113FDB5C),
])
def test_crc32c_known_answers(data, want):
    assert tfckpt.crc32c(data) == want


def test_mask_is_rotate_plus_delta():
    assert tfckpt.mask_crc(0) == 0xA282EAD8
    c = 0x12345678
    assert tfckpt.mask_crc(c) == ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def test_snappy_hand_assembled():
    # len 12; literal "abc" (tag (3-1)<<2); copy-1 len 9 off 3 (tag (9-4)<<2 | 1)
    assert tfckpt.snappy_decompress(bytes([12, 0x08]) + b"abc" + bytes([0x15, 0x03])) == b"abc" * 4
    # copy-2: len 6 off 2 over "xy" -> overlapping copy
    assert tfckpt.snappy_decompress(bytes([8, 0x04]) + b"xy" + bytes([(6 - 1) << 2 | 2, 2, 0])) == b"xy" * 4
    # 61-byte literal needs the 1-extra-byte length form (tag 60 << 2)
    lit = bytes(range(61))
    assert tfckpt.snappy_decompress(bytes([61, 60 << 2, 60]) + lit) == lit
    with pytest.raises(tfckpt.CheckpointError):
        tfckpt.snappy_decompress(bytes([4, 0x0d, 0x05]))     # copy before any output


def _blk(contents, ctype=0):
    tail = bytes([ctype])
    return contents + tail + struct.pack("<I", tfckpt.mask_crc(tfckpt.crc32c(contents + tail)))


def _hand_table(compress=False):
    """Two-entry data block with prefix compression, empty meta block, one-entry index."""
    data = (bytes([0, 1, 1]) + b"a1" +            # shared 0, key "a", value "1"
            bytes([1, 1, 2]) + b"b22" +           # shared 1 -> key "ab", value "22"
            struct.pack("<II", 0, 1))
    stored = data
    if compress:                                   # one snappy literal
        stored = bytes([len(data), (len(data) - 1) << 2]) + data
    out = _blk(stored, 1 if compress else 0)
    h_data = bytes([0, len(stored)])
    meta = struct.pack("<II", 0, 1)
    h_meta = bytes([len(out), len(meta)])
    out += _blk(meta)
    index = bytes([0, 2, 2]) + b"ab" + h_data + struct.pack("<II", 0, 1)
    h_index = bytes([len(out), len(index)])
    out += _blk(index)
    foot = h_meta + h_index
    return out + foot + bytes(40 - len(foot)) + struct.pack("<Q", 0xdb4775248b80fb57)


@pytest.mark.parametrize("compress", [False, True])
def test_read_hand_assembled_table(compress):
    assert tfckpt.read_table(_hand_table(compress)) == [(b"a", b"1"), (b"ab", b"22")]


def test_table_writer_matches_hand_layout():
    assert tfckpt.write_table([(b"a", b"1"), (b"ab", b"22")]) == _hand_table()


def test_table_detects_corruption():
    t = bytearray(_hand_table())
    t[4] ^= 0x01
    with pytest.raises(tfckpt.CheckpointError, match="checksum"):
        tfckpt.read_table(bytes(t))
    t = bytearray(_hand_table())
    t[-1] ^= 0xFF
    with pytest.raises(tfckpt.CheckpointError, match="magic"):
        tfckpt.read_table(bytes(t))


def test_large_table_many_blocks_roundtrip():
    rng = np.random.default_rng(0)
    keys = sorted({("scope_%03d/var_%d" % (rng.integers(1000), i)).encode() for i in range(700)})
    ents = [(k, rng.bytes(int(rng.integers(0, 40)))) for k in keys]
    img = tfckpt.write_table(ents, block_size=512)
    assert tfckpt.read_table(img) == ents


def test_entry_proto_fields():
    msg = tfckpt.encode_entry(1, (22, 20), 0, 1760, 1760, 0xDEADBEEF)
    # dtype=1 varint, shape dims {size=22}{size=20}, offset, size, fixed32 crc
    assert msg[:2] == bytes([0x08, 0x01])
    assert msg[2:12] == bytes([0x12, 0x08, 0x12, 0x02, 0x08, 22, 0x12, 0x02, 0x08, 20])
    e = tfckpt.decode_entry(msg)
    assert (e["dtype"], e["shape"], e["offset"], e["size"], e["crc32c"]) == (1, [22, 20], 1760, 1760, 0xDEADBEEF)
    h = tfckpt.decode_header(tfckpt.encode_header(1))
    assert (h["num_shards"], h["endianness"], h["producer"]) == (1, 0, 1)


def test_bundle_roundtrip_and_tamper(tmp_path):
    rng = np.random.default_rng(1)
    t = {"phi_E_O1/r1_w1o": rng.standard_normal((4, 20)).astype(np.float32),
         "map_conv/map_theta1": rng.standard_normal((1, 2, 1, 1)).astype(np.float32),
         "beta1_power": np.float32(0.729).reshape(()),
         "global_step": np.int64(7).reshape(()),
         "d": rng.standard_normal(5)}
    pre = str(tmp_path / "g2g.model-3")
    tfckpt.write(pre, t)
    r = tfckpt.read(pre)
    assert set(r) == set(t)
    for k in t:
        assert r[k].dtype == np.asarray(t[k]).dtype and r[k].shape == np.asarray(t[k]).shape
        np.testing.assert_array_equal(r[k], t[k])
    with open(pre + ".data-00000-of-00001", "r+b") as f:
        f.seek(3)
        b = f.read(1)
        f.seek(3)
        f.write(bytes([b[0] ^ 0x40]))
    with pytest.raises(tfckpt.CheckpointError, match="checksum"):
        tfckpt.read(pre)


@pytest.mark.parametrize("v", [1, 2, 3, 4])
def test_engine_state_tf_names(v, tmp_path):
    rng = np.random.default_rng(v)
    n = layout.n_params(v)
    flat, m, vv = (rng.standard_normal(n).astype(np.float32) for _ in range(3))
    bp = np.array([0.9 ** 4, 0.999 ** 4], np.float32)
    pre = str(tmp_path / "g2g.model-1")
    tfckpt.write(pre, tfckpt.state_tensors(flat, v, m, vv, bp))
    tens = tfckpt.read(pre)
    names = [s.split(":")[0] for s, _ in layout.specs(v)]
    assert set(tens) == set(names) | {x + "/Adam" for x in names} | \
        {x + "/Adam_1" for x in names} | {"beta1_power", "beta2_power"}
    f2, m2, v2, bp2 = tfckpt.engine_state(tens, v)
    for a, b in ((f2, flat), (m2, m), (v2, vv), (bp2, bp)):
        np.testing.assert_array_equal(a, b)
    # a reference-style checkpoint (Saver built before the optimizer): weights only
    ref = {k: tens[k] for k in names}
    f3, m3, _, _ = tfckpt.engine_state(ref, v)
    np.testing.assert_array_equal(f3, flat)
    assert m3 is None
    ref.pop(names[0])
    with pytest.raises(tfckpt.CheckpointError, match="lacks"):
        tfckpt.engine_state(ref, v)
    bad = dict(tens)
    bad[names[-1]] = np.zeros((2, 1, 1, 1), np.float32)
    with pytest.raises(tfckpt.CheckpointError, match="shape"):
        tfckpt.engine_state(bad, v)


def test_checkpoint_state_file(tmp_path):
    tfckpt.write_state_file(str(tmp_path), "g2g.model-12")
    assert tfckpt.latest(str(tmp_path)) == "g2g.model-12"
    (tmp_path / "checkpoint").write_text(
        'model_checkpoint_path: "./checkpoint40/glide/glide/model_2/2/g2g.model-5"\n'
        'all_model_checkpoint_paths: "./checkpoint40/glide/glide/model_2/2/g2g.model-5"\n')
    assert tfckpt.latest(str(tmp_path)) == "g2g.model-5"
    assert tfckpt.latest(str(tmp_path / "nope")) is None


def test_native_crc32c_matches_table_loop():
    """libhdgnn's slicing-by-8 CRC-32C (hdg_crc32c) = the reference table loop, at every
    length mod 8 and with a running crc; the standard check value of "123456789"."""
    import random
    from hdgnn import _lib
    lib = _lib.load()
    rng = random.Random(7)
    for n in (0, 1, 3, 7, 8, 9, 15, 16, 17, 255, 4096, 4099):
        data = bytes(rng.getrandbits(8) for _ in range(n))
        for c0 in (0, 0xDEADBEEF):
            assert lib.hdg_crc32c(data, n, c0) == tfckpt.crc32c_py(data, c0)
    assert lib.hdg_crc32c(b"123456789", 9, 0) == 0xE3069283
    assert tfckpt.crc32c(b"123456789") == 0xE3069283


def test_background_saver_keeps_order_and_state(tmp_path):
    """graph2graph.train saves every epoch in the background (Saver.save(background=True)):
    each bundle holds the state at its save() call even when the engine's tensors change
    before the writer thread runs, max_to_keep and the state file behave as Saver.save's."""
    import types

    import torch

    from hdgnn.model import Saver
    v = 2
    flat = layout.init_flat(3, v).astype(np.float32)
    P, so = flat.size, layout.state_offsets(v)      # Engine.state's layout, on the host
    state = torch.zeros(so["len"])
    eng = types.SimpleNamespace(state=state, params=state[:P], m=state[so["m"]:so["m"] + P],
                                v=state[so["v"]:so["v"] + P],
                                beta_pow=state[so["beta_pow"]:so["beta_pow"] + 2])
    eng.params.copy_(torch.from_numpy(flat))
    eng.beta_pow.copy_(torch.tensor([0.9, 0.999]))
    sv = Saver(types.SimpleNamespace(engine=eng, variant=v))
    want = {}
    for step in range(1, 8):
        eng.params += 1.0               # the "next epoch" runs while the bundle is written
        eng.m.fill_(step)
        want[step] = (eng.params.numpy().copy(), float(step))
        sv.save(None, str(tmp_path / "g2g.model"), global_step=step, background=True)
    sv.flush()
    assert tfckpt.latest(str(tmp_path)) == "g2g.model-7"
    for step in range(1, 8):
        present = (tmp_path / ("g2g.model-%d.index" % step)).exists()
        assert present == (step >= 3)                       # newest 5 kept
        if present:
            fl, m, _, bp = tfckpt.engine_state(tfckpt.read(str(tmp_path / ("g2g.model-%d" % step))), v)
            np.testing.assert_array_equal(fl, want[step][0])
            assert np.all(m == want[step][1])
            np.testing.assert_array_equal(bp, np.float32([0.9, 0.999]))


def test_native_bundle_template_bytes_equal_python_writer(tmp_path):
    """tfckpt.BundleTemplate (libhdgnn hdg_bundle_write: the saver thread's GIL-free path)
    writes the same .index / .data bytes as the Python encoder, for every variant, and the
    bundle reads back to the state it was given."""
    for v in (1, 2, 3, 4):
        P = layout.n_params(v)
        so = layout.state_offsets(v)              # Engine.state: 64-byte aligned slices
        st = np.random.default_rng(v).standard_normal(so["len"]).astype(np.float32)
        sm, sv, sb = st[so["m"]:so["m"] + P], st[so["v"]:so["v"] + P], st[so["beta_pow"]:]
        t = tfckpt.BundleTemplate(v)
        for rep in range(2):                 # the template is reused across saves
            st += np.float32(rep)
            t.write(str(tmp_path / ("n%d" % v)), st)
            tfckpt.write(str(tmp_path / ("p%d" % v)), tfckpt.state_tensors(st[:P], v, sm, sv, sb))
            for ext in (".index", ".data-00000-of-00001"):
                assert (tmp_path / ("n%d%s" % (v, ext))).read_bytes() == \
                    (tmp_path / ("p%d%s" % (v, ext))).read_bytes()
            fl, m, vv, bp = tfckpt.engine_state(tfckpt.read(str(tmp_path / ("n%d" % v))), v)
            np.testing.assert_array_equal(np.concatenate([fl, m, vv, bp]),
                                          np.concatenate([st[:P], sm, sv, sb]))
        assert not list(tmp_path.glob("*.tmp"))   # written under .tmp names, renamed in place
    with pytest.raises(tfckpt.CheckpointError):
        tfckpt.BundleTemplate(2).write(str(tmp_path / "bad"), np.zeros(5, np.float32))


def test_native_bundle_write_checks_gather_bounds(tmp_path):
    """hdg_bundle_write bounds-checks every gather index against n_state itself (not only
    the Python wrapper's size check) and leaves no file behind when it refuses."""
    import ctypes
    from hdgnn import _lib
    lib = _lib.load()
    t = tfckpt.BundleTemplate(2)
    st = np.zeros(t.n_state, np.float32)
    gather = t.gather.copy()
    gather[7] = t.n_state                     # one past the end
    img = t.image.copy()
    prefix = str(tmp_path / "oob")
    rc = lib.hdg_bundle_write((prefix + ".data-00000-of-00001").encode(),
                              (prefix + ".index").encode(), st.ctypes.data, st.size,
                              gather.ctypes.data, gather.size, img.ctypes.data, img.size,
                              t.entries.ctypes.data, len(t.entries), t.blocks.ctypes.data,
                              len(t.blocks))
    assert rc == 1000                          # HDG_EINVAL
    assert b"gather" in lib.hdg_last_error()
    assert not list(tmp_path.iterdir())


def test_native_writer_order_text_and_errors(tmp_path):
    """tfckpt.BundleWriter (libhdgnn's writer thread): jobs run in submission order (a
    bundle, then its removals, then the state file; appended text accumulates), and a
    failure surfaces at the next flush() -- once -- without stopping later jobs."""
    t = tfckpt.BundleTemplate(2)
    w = tfckpt.BundleWriter(t)
    st = np.arange(t.n_state, dtype=np.float32)
    res = str(tmp_path / "result_2.npy")
    for k in range(3):
        w.submit(str(tmp_path / ("m-%d" % k)), st + k,
                 removes=[str(tmp_path / ("m-%d.index" % (k - 2)))] if k >= 2 else (),
                 text_path=str(tmp_path / "checkpoint"), text="latest %d\n" % k)
        w.submit(text_path=res, text="Epoch %d\n" % (k + 1), append=True)
    w.flush()
    assert open(res).read() == "Epoch 1\nEpoch 2\nEpoch 3\n"
    assert open(tmp_path / "checkpoint").read() == "latest 2\n"
    assert not (tmp_path / "m-0.index").exists() and (tmp_path / "m-1.index").exists()
    fl, m, v, bp = tfckpt.engine_state(tfckpt.read(str(tmp_path / "m-2")), 2)
    P, so = layout.n_params(2), layout.state_offsets(2)
    np.testing.assert_array_equal(fl, (st + 2)[:P])
    np.testing.assert_array_equal(m, (st + 2)[so["m"]:so["m"] + P])
    w.submit(str(tmp_path / "missing_dir" / "x"), st)       # cannot be written
    w.submit(text_path=res, text="after\n", append=True)     # still runs
    with pytest.raises(tfckpt.CheckpointError, match="missing_dir"):
        w.flush()
    w.flush()                                                 # reported once
    assert open(res).read().endswith("Epoch 3\nafter\n")
    w.close()


def test_background_saver_failure_surfaces_at_next_save(tmp_path):
    """A background bundle write that fails (here: its .tmp data path is a directory) is
    reported by the next save() -- not only at the end of training -- and the keep-list is
    re-booked from the files on disk: the failed prefix is not listed in the state file, and
    the older bundle that the failed job would have removed is removed by a later save."""
    import time
    import types

    import torch

    from hdgnn.model import Saver
    v = 2
    so = layout.state_offsets(v)
    eng = types.SimpleNamespace(state=torch.zeros(so["len"]))
    sv = Saver(types.SimpleNamespace(engine=eng, variant=v), max_to_keep=2)
    pre = str(tmp_path / "g2g.model")
    st = np.zeros(so["len"], np.float32)
    for step in (1, 2):
        sv.save(None, pre, global_step=step, background=True, state=st + step)
    sv.flush()
    # step 3 cannot be written; its job would have removed bundle 1
    os.makedirs(pre + "-3.data-00000-of-00001.tmp")
    sv.save(None, pre, global_step=3, background=True, state=st + 3)
    with pytest.raises(tfckpt.CheckpointError):
        sv.flush()
    assert not os.path.exists(pre + "-3.index")
    assert os.path.exists(pre + "-1.index")    # the failed job stopped before its removals
    assert sv._last == [pre + "-1", pre + "-2"]
    sv.save(None, pre, global_step=4, background=True, state=st + 4)
    sv.flush()
    assert not os.path.exists(pre + "-1.index")   # re-booked: removed now
    assert os.path.exists(pre + "-2.index") and os.path.exists(pre + "-4.index")
    assert tfckpt.latest(str(tmp_path)) == "g2g.model-4"
    assert "g2g.model-3" not in open(tmp_path / "checkpoint").read()
    # the next save() itself raises a failed background job's error (no flush needed)
    os.makedirs(pre + "-5.data-00000-of-00001.tmp")
    sv.save(None, pre, global_step=5, background=True, state=st + 5)
    time.sleep(1.0)                            # the writer thread reaches the failure
    with pytest.raises(tfckpt.CheckpointError):
        sv.save(None, pre, global_step=6, background=True, state=st + 6)
    assert sv._last == [pre + "-2", pre + "-4"]
    sv.flush()
