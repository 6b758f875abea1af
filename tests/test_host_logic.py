"""Host-side logic of polar_code_amd against the reference's golden vectors (no GPU)."""
import numpy as np
import pytest

from polar_code_amd import config
from polar_code_amd.polar import crc as pcrc
from polar_code_amd.polar import polar as ppolar
from polar_code_amd.utils.seeding import seed_all


def test_config_defaults():
    cfg = config.get_config()
    assert (cfg.N, cfg.K, cfg.crc_poly, cfg.crc_bits, cfg.retries) == (128, 64, "0x1864CFB", 24, 8)
    assert cfg.list_sizes == [1, 2, 4, 8] and cfg.ebno_sweep == [4.0, 6.5, 0.5]


def test_info_sets(golden):
    g = golden("g1_info_sets.npz")
    for key in g.files:
        _, N, K = key.split("_")
        np.testing.assert_array_equal(ppolar.construct_info_set(int(N), int(K)), g[key])
    with pytest.raises(ValueError):
        ppolar.construct_info_set(100, 10)
    with pytest.raises(ValueError):
        ppolar.construct_info_set(128, 0)


def test_crc_attach_check(golden):
    g = golden("g2_crc.npz")
    np.testing.assert_array_equal(pcrc.attach_crc(g["payload"], "0x1864CFB"), g["attached"])
    for p, a in zip(g["payload"][:16], g["attached"][:16]):
        np.testing.assert_array_equal(pcrc.attach_crc(p, "0x1864CFB"), a)
    np.testing.assert_array_equal(pcrc.attach_crc(g["payload8"], "0x17"), g["attached8_0x17"])
    np.testing.assert_array_equal(pcrc.check_crc(g["attached"], "0x1864CFB"), g["check_ok"])
    np.testing.assert_array_equal(pcrc.check_crc(g["corrupted"], "0x1864CFB"), g["check_bad"])
    np.testing.assert_array_equal(pcrc.check_crc(g["random64"], "0x1864CFB"), g["check_random"])
    assert pcrc.check_crc(g["attached"][0], "0x1864CFB") is True
    with pytest.raises(ValueError):
        pcrc.check_crc(np.zeros(24, np.int8), "0x1864CFB")
    with pytest.raises(ValueError):
        pcrc.attach_crc(np.zeros(4, np.int8), "")
    with pytest.raises(ValueError):
        pcrc.attach_crc(np.zeros(4, np.int8), "0x1")


def test_crc_roundtrip_reference_case():
    # tests/test_scl_crc.py:25-37 of the reference, restated
    seed_all(7)
    msg = np.random.randint(0, 2, size=40, dtype=np.int8)
    msg_crc = pcrc.attach_crc(msg, "0x1864CFB")
    assert msg_crc.shape[0] == 64 and pcrc.check_crc(msg_crc, "0x1864CFB")
    corrupted = msg_crc.copy()
    corrupted[3] ^= 1
    assert not pcrc.check_crc(corrupted, "0x1864CFB")


def test_encode(golden):
    g = golden("g3_encode.npz")
    np.testing.assert_array_equal(ppolar.encode(g["msg"]), g["code"])
    np.testing.assert_array_equal(ppolar.encode(g["msg"][0]), g["code"][0])
    np.testing.assert_array_equal(ppolar._polar_transform(g["u"]), g["transform"])
    with pytest.raises(ValueError):
        ppolar.encode(np.zeros(10, np.int8))


def test_f_g_helpers():
    a = np.array([1.0, -2.0, 0.0, -0.5])
    b = np.array([-3.0, -1.0, 5.0, 0.25])
    np.testing.assert_array_equal(ppolar._f(a, b), [-1.0, 1.0, 0.0, -0.25])
    np.testing.assert_array_equal(ppolar._g(a, b, np.array([0, 1, 1, 0], np.int8)), [-2.0, 1.0, 5.0, -0.25])


def test_philox_stream_ids_distinct_on_fine_grids():
    """--rng philox: every SNR point of a grid gets its own Philox stream (0.1 dB points keep
    their historical word round(10 Eb/N0); finer grids no longer collide)."""
    from polar_code_amd.utils.seeding import philox_stream_id

    assert [philox_stream_id(x) for x in (4.0, 4.5, 5.0, 6.5)] == [40, 45, 50, 65]
    for step in (0.05, 0.01, 0.25, 0.125):
        grid = np.round(np.arange(3.0, 7.0 + 1e-9, step), 6)
        ids = [philox_stream_id(x) for x in grid]
        assert len(set(ids)) == len(ids), step
        assert all(0 <= i < 2 ** 32 for i in ids)
    # negative grid points keep their historical 32-bit words (round(10 x) & 0xFFFFFFFF)
    assert [philox_stream_id(x) for x in (-1.0, -0.5, -2.0)] == [0xFFFFFFF6, 0xFFFFFFFB, 0xFFFFFFEC]
    # grids spanning negative and positive points, coarse and fine: no shared stream, and no
    # off-grid word equals any grid word
    for step in (0.1, 0.05, 0.01, 0.001):
        grid = np.round(np.arange(-3.0, 3.0 + 1e-9, step), 6)
        ids = [philox_stream_id(x) for x in grid]
        assert len(set(ids)) == len(ids), step
    on = {philox_stream_id(k / 10) for k in range(-2000, 2001)}
    off = {philox_stream_id(x) for x in (-1e-6, -0.05, 0.05, -123.456789, 7.77)}
    assert not (on & off)


def test_closed_decoder_raises_clearly():
    """A Decoder closed by close() or release_decoders() (get_decoder results are shared) raises a
    clear RuntimeError on use instead of passing a NULL handle to the library; set_pipelined
    rejects depths outside 1..4 in Python."""
    import pytest

    from polar_code_amd import _native

    d = object.__new__(_native.Decoder)  # (no GPU here: a handle-less object, as after close())
    d._hraw = None
    assert d.closed
    for call in (lambda: d.join(), lambda: d.set_pipelined(True), lambda: d.handle, lambda: d.sync()):
        with pytest.raises(RuntimeError, match="closed"):
            call()
    d.close()  # idempotent
    d._hraw = object()  # (a stand-in handle: the depth check runs before any library call)
    for depth in (0, 5, -1):
        with pytest.raises(ValueError, match="depth"):
            d.set_pipelined(True, depth=depth)
    d._hraw = None
