"""The dbfarm loader: BBP.dir entries (host parsing, CPU) and heaps streamed
into HBM (GPU), against a bat directory written in the reference's format."""
import numpy as np
import pytest

from dbfarm_writer import physical, props, write_dbfarm


def test_physical_names():
    # BBPgetfilename: octal, 2-digit octal subdirectories above 0100
    assert physical(5) == "5"
    assert physical(0o1234) == "12/1234"
    assert physical(0o123456) == "12/34/123456"


def _farm(tmp_path):
    r = np.random.default_rng(5)
    bats = [
        {"id": 3, "name": "sys_lineitem_l_quantity", "type": "lng",
         "values": r.integers(1, 51, 100_003).astype(np.int64) * 100, "props": props(nonil=True)},
        {"id": 0o1234, "name": "sys_lineitem_l_shipdate", "type": "int", "values": r.integers(0, 10**6, 5000).astype(np.int32),
         "hseqbase": 0, "props": 0},
        {"id": 0o123456, "name": "sys_lineitem_l_returnflag", "type": "str",
         "strings": [["A", "N", "R"][i % 3] for i in range(3001)]},
        {"id": 9, "name": "sys_dense", "type": "void", "count": 77, "tseqbase": 1000},
        {"id": 10, "name": "sys_empty", "type": "lng", "values": np.zeros(0, np.int64), "props": 0},
    ]
    write_dbfarm(str(tmp_path), bats)
    return bats


def test_bbpdir_parse(tmp_path):
    # host-side parsing only: no device needed
    from monetdb_amd import gdk
    bats = _farm(tmp_path)
    ents = gdk.BBPreaddir(str(tmp_path / "BBP.dir"))
    assert [e.batid for e in ents] == [b["id"] for b in bats]
    e = ents[0]
    assert e.name == b"sys_lineitem_l_quantity" and e.type == b"lng" and e.count == 100_003
    assert e.tail == b"3.tail" and e.props & 0x400
    assert ents[1].tail == b"12/1234.tail"
    assert ents[2].tail == b"12/34/123456.tail1" and ents[2].theap == b"12/34/123456.theap" and ents[2].var
    assert ents[3].type == b"void" and ents[3].tseqbase == 1000
    assert ents[4].count == 0 and not (tmp_path / "12.tail").exists()


def test_bbpdir_version(tmp_path):
    # gdk_bbp.c:990-998: a BBP.dir of another library version is refused
    from monetdb_amd import gdk
    from dbfarm_writer import GDKLIBRARY
    bats = [{"id": 3, "name": "x", "type": "lng", "values": np.arange(3, dtype=np.int64)}]
    for v, word in ((GDKLIBRARY + 1, "newer"), (0o61047, "too old")):
        write_dbfarm(str(tmp_path), bats, version=v)
        with pytest.raises(gdk.GDKError, match=word):
            gdk.BBPreaddir(str(tmp_path / "BBP.dir"))


@pytest.mark.gpu
def test_batload(gdk, tmp_path):
    bats = _farm(tmp_path)
    ents = gdk.BBPreaddir(str(tmp_path / "BBP.dir"))
    q = gdk.BATload(str(tmp_path), ents[0])
    assert np.array_equal(q.to_numpy(), bats[0]["values"]) and q.s.tnonil == 1
    d = gdk.BATload(str(tmp_path), ents[1])
    assert np.array_equal(d.to_numpy(), bats[1]["values"])
    s = gdk.BATload(str(tmp_path), ents[2])
    assert s.count() == 3001 and s.s.twidth == 1
    # the string heap came along: group the offsets -> 3 groups in A, N, R order
    g, e, h = gdk.BATgroup(s)
    assert e.count() == 3 and list(h.to_numpy()) == [1001, 1000, 1000]
    v = gdk.BATload(str(tmp_path), ents[3])
    assert v.ttype == gdk.TYPE_void and list(v.to_numpy()[:3]) == [1000, 1001, 1002]
    # a loaded column feeds the operators: thetaselect on the loaded lng
    sel = gdk.BATthetaselect(q, None, 2400, "<")
    assert sel.count() == int((bats[0]["values"] < 2400).sum())
    # an empty persistent BAT has no tail file (HEAPsave wrote none)
    z = gdk.BATload(str(tmp_path), ents[4])
    assert z.count() == 0 and z.ttype == gdk.TYPE_lng
