"""Yjs ``workflows`` output map (C02): the update v1 byte layout pinned from the Yjs/lib0 format
(y_py is not importable here, so byte parity with y_py itself is unpinned), overwrite history
(origin + ContentDeleted + delete set), decode round trip, and the server/executor hook."""
import base64
import json

from comfy_gen_server_amd.api import ymap


def _vs(s):
    b = s.encode()
    return [len(b)] + list(b)


def test_first_set_layout():
    d = ymap.YDoc(client_id=1)
    d.get_map("workflows").set("a", "x")
    got = list(d.encode_state_as_update())
    want = ([1, 1, 1, 0,                    # 1 client, 1 struct, client 1, first clock 0
             0x28, 1] + _vs("workflows") + _vs("a") +   # Item: ContentAny | parentSub; root parent + key
            [1, 119] + _vs("x") +           # ContentAny: 1 value, string tag 119
            [0])                            # empty delete set
    assert got == want


def test_overwrite_layout_and_delete_set():
    d = ymap.YDoc(client_id=300)            # multi-byte varuint client id
    m = d.get_map("workflows")
    m.set("a", "x")
    m.set("a", "y")
    got = list(d.encode_state_as_update())
    cid = [0xAC, 0x02]                      # 300 as a lib0 varuint
    want = ([1, 2] + cid + [0,
            0x21, 1] + _vs("workflows") + _vs("a") + [1] +      # deleted first value: ContentDeleted(1)
            [0xA8] + cid + [0] + [1, 119] + _vs("y") +           # origin (300, 0), parentSub bit, Any "y"
            [1] + cid + [1, 0, 1])                               # delete set: client 300, [clock 0, len 1]
    assert got == want


def test_roundtrip_and_values():
    d = ymap.YDoc(client_id=7)
    m = d.get_map("workflows")
    vals = {"img": json.dumps([[1, 2], [3, 4]]), "n": 42, "f": 0.5, "neg": -70000, "big": 2 ** 40, "t": True,
            "none": None, "obj": {"k": [1, "two"]}, "uni": "héllo ✓"}
    for k, v in vals.items():
        m.set(k, v)
    m.set("n", 43)
    dec = ymap.decode_update(d.encode_state_as_update())
    state = dec["maps"]["workflows"]
    exp = dict(vals, n=43)
    assert state.keys() == exp.keys()
    for k, v in exp.items():
        assert state[k] == v, (k, state[k], v)
    assert dec["deletes"] == {7: [(1, 1)]}
    assert m.to_json() == exp
    # incremental update from a state vector: only the new struct(s), whole delete set
    inc = ymap.decode_update(d.encode_state_as_update(since=len(vals)))
    assert len(inc["structs"]) == 1 and inc["structs"][0]["value"] == 43


def test_output_map_broadcast_payload():
    om = ymap.OutputMap(client_id=5)
    om.set("final", json.dumps({"images": 1}))
    msg = om.encode_update()
    assert msg["encoding"] == "yjs-update-v1" and msg["map"] == "workflows"
    dec = ymap.decode_update(base64.b64decode(msg["update"]))
    assert dec["maps"]["workflows"]["final"] == json.dumps({"images": 1})
    assert om.get("final") == json.dumps({"images": 1})
