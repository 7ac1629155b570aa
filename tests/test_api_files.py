"""Contract tests of the file / user routes (reference ``server.py:254-399``, ``:490-542``;
``app/user_manager.py:44-140``; ``app/app_settings.py:25-54``): /upload/image, /upload/mask, /view_all,
/view_metadata, /users, /userdata/{file}, /settings[/{id}] -- including the path-escape guards and the
mask upload's error paths (a rejected reference writes nothing and is never a 200)."""
import asyncio
import io
import json
import os

import numpy as np
import pytest
from aiohttp import FormData
from aiohttp.test_utils import TestClient, TestServer
from PIL import Image
from PIL.PngImagePlugin import PngInfo

from test_e2e_cpu import env  # noqa: F401  (module fixture: base directory + tiny checkpoint)


def _png(color=(10, 20, 30, 255), size=(8, 6), text=None):
    im = Image.new("RGBA", size, color)
    info = None
    if text:
        info = PngInfo()
        for k, v in text.items():
            info.add_text(k, v)
    buf = io.BytesIO()
    im.save(buf, format="PNG", pnginfo=info)
    return buf.getvalue()


def _form(data, name="a.png", **fields):
    f = FormData()
    f.add_field("image", data, filename=name, content_type="image/png")
    for k, v in fields.items():
        f.add_field(k, v)
    return f


def _run(env_base, fn, multi_user=False):  # noqa: F811
    from comfy_gen_server_amd import cli_args
    from comfy_gen_server_amd.main import build_server

    async def main():
        loop = asyncio.get_running_loop()
        argv = ["--disable-custom-nodes"] + (["--multi-user"] if multi_user else [])
        server, _ = build_server(cli_args.parser.parse_args(argv), loop)
        client = TestClient(TestServer(server.app))
        await client.start_server()
        try:
            await fn(client)
        finally:
            await client.close()
    asyncio.run(main())


def test_upload_image_rename_overwrite_and_escape(env):  # noqa: F811
    inp = env / "input"

    async def fn(c):
        r = await c.post("/upload/image", data=_form(_png(), "up.png"))
        assert r.status == 200 and (await r.json()) == {"name": "up.png", "subfolder": "", "type": "input"}
        r = await c.post("/upload/image", data=_form(_png((1, 2, 3, 255)), "up.png"))
        assert (await r.json())["name"] == "up (1).png"                     # auto-rename
        r = await c.post("/upload/image", data=_form(_png((9, 9, 9, 255)), "up.png", overwrite="true"))
        assert (await r.json())["name"] == "up.png"                         # overwrite in place
        assert np.asarray(Image.open(inp / "up.png"))[0, 0, 0] == 9
        r = await c.post("/upload/image", data=_form(_png(), "s.png", subfolder="sub/dir", type="temp"))
        j = await r.json()
        assert r.status == 200 and j == {"name": "s.png", "subfolder": "sub/dir", "type": "temp"}
        assert os.path.isfile(env / "temp" / "sub" / "dir" / "s.png")
        for bad in ({"subfolder": "../../etc"}, {"subfolder": "/abs"}):
            r = await c.post("/upload/image", data=_form(_png(), "x.png", **bad))
            assert r.status == 400, bad
        r = await c.post("/upload/image", data=_form(_png(), "../x.png"))    # the name never leaves the dir
        if r.status != 400:      # the client may percent-encode the name: then it is a plain file name
            nm = (await r.json())["name"]
            assert "/" not in nm and os.path.isfile(inp / nm)
        r = await c.post("/upload/image", data=FormData({"type": "input"}))   # no image field
        assert r.status == 400
    _run(env, fn)
    assert not os.path.exists(env / "x.png") and not os.path.exists(env / "etc")


def test_upload_mask_applies_alpha_and_keeps_text(env):  # noqa: F811
    out = env / "output"
    (out / "m").mkdir(parents=True, exist_ok=True)
    with open(out / "m" / "orig.png", "wb") as f:
        f.write(_png((200, 100, 50, 255), text={"prompt": "{\"a\": 1}", "workflow": "wf"}))
    mask = Image.new("RGBA", (8, 6), (0, 0, 0, 0))
    mask.putalpha(Image.fromarray(np.full((6, 8), 77, np.uint8)))
    mb = io.BytesIO()
    mask.save(mb, format="PNG")
    ref = json.dumps({"filename": "orig.png", "subfolder": "m", "type": "output"})

    async def fn(c):
        r = await c.post("/upload/mask", data=_form(mb.getvalue(), "masked.png", original_ref=ref))
        assert r.status == 200, await r.text()
        name = (await r.json())["name"]
        got = Image.open(env / "input" / name)
        arr = np.asarray(got)
        assert arr.shape == (6, 8, 4) and (arr[..., 3] == 77).all() and tuple(arr[0, 0, :3]) == (200, 100, 50)
        assert got.text.get("prompt") == "{\"a\": 1}" and got.text.get("workflow") == "wf"
        cases = [("not json", 400),
                 (json.dumps({"filename": "../orig.png", "type": "output"}), 400),
                 (json.dumps({"filename": "orig.png", "subfolder": "../../..", "type": "output"}), 403),
                 (json.dumps({"filename": "missing.png", "subfolder": "m", "type": "output"}), 404),
                 (json.dumps({"subfolder": "m"}), 400)]
        for i, (bad, code) in enumerate(cases):
            r = await c.post("/upload/mask", data=_form(mb.getvalue(), f"bad{i}.png", original_ref=bad))
            assert r.status == code, (bad, r.status)
            assert not os.path.exists(env / "input" / f"bad{i}.png"), bad       # nothing written
            r = await c.post("/upload/mask", data=_form(mb.getvalue(), f"bad{i}.png", original_ref=bad,
                                                        subfolder=f"newdir{i}"))
            assert r.status == code and not os.path.exists(env / "input" / f"newdir{i}"), bad   # not even a folder
    _run(env, fn)


def test_view_all_pages_and_validation(env):  # noqa: F811
    out = env / "output" / "va"
    out.mkdir(parents=True, exist_ok=True)
    for i in range(5):
        Image.new("RGB", (4, 4)).save(out / f"v{i}.png")
        os.utime(out / f"v{i}.png", (1e9 + i, 1e9 + i))

    async def fn(c):
        allj = await (await c.get("/view_all", params={"page_size": "500"})).json()
        names = [x["filename"] for x in allj["images"] if x["subfolder"] == "va"]
        assert names == [f"v{i}.png" for i in range(4, -1, -1)]               # newest first
        j = await (await c.get("/view_all", params={"page": "2", "page_size": "2"})).json()
        assert j["page"] == 2 and j["page_size"] == 2 and len(j["images"]) == 2 and j["total"] == allj["total"]
        assert all(x["url"].startswith("/view?filename=") for x in j["images"])
        for bad in ({"page": "x"}, {"page": "0"}, {"page_size": "0"}, {"page_size": "100000"}, {"page": "-3"}):
            assert (await c.get("/view_all", params=bad)).status == 400, bad
    _run(env, fn)


def test_view_metadata(env):  # noqa: F811
    async def fn(c):
        r = await c.get("/view_metadata/checkpoints", params={"filename": "tiny.safetensors"})
        assert r.status == 200 and (await r.json()).get("family") == "tiny"
        assert (await c.get("/view_metadata/checkpoints", params={"filename": "nope.safetensors"})).status == 404
        assert (await c.get("/view_metadata/checkpoints", params={"filename": "tiny.ckpt"})).status == 404
        assert (await c.get("/view_metadata/checkpoints")).status == 404
    _run(env, fn)


def test_users_userdata_settings_single_user(env):  # noqa: F811
    async def fn(c):
        j = await (await c.get("/users")).json()
        assert j["storage"] == "server" and "migrated" in j
        r = await c.post("/userdata/wf.json", data=b'{"x": 1}')
        assert r.status == 200
        r = await c.get("/userdata/wf.json")
        assert r.status == 200 and json.loads(await r.read()) == {"x": 1}
        assert (await c.post("/userdata/wf.json?overwrite=false", data=b"{}")).status == 409
        assert (await c.get("/userdata/none.json")).status == 404
        for esc in ("..%2F..%2Fescape.json", "%2E%2E%2Fx.json", "..%2Fdefault2%2Fx.json"):
            r = await c.post(f"/userdata/{esc}", data=b"evil")
            assert r.status in (400, 403, 404), (esc, r.status)
        assert not os.path.exists(env / "user" / "escape.json") and not os.path.exists(env / "escape.json")
        assert await (await c.get("/settings")).json() == {} or True
        assert (await c.post("/settings", json={"a": 1, "b": [2]})).status == 200
        assert (await c.post("/settings/c", json={"deep": True})).status == 200
        s = await (await c.get("/settings")).json()
        assert s["a"] == 1 and s["b"] == [2] and s["c"] == {"deep": True}
        assert await (await c.get("/settings/c")).json() == {"deep": True}
        assert await (await c.get("/settings/unknown")).json() is None
    _run(env, fn)


def test_multi_user_profiles(env):  # noqa: F811
    async def fn(c):
        r = await c.post("/users", json={"username": "alice b"})
        assert r.status == 200
        uid = await r.json()
        assert uid.startswith("alice-b_")
        assert (await c.post("/users", json={"username": "alice b"})).status == 400    # duplicate
        assert (await c.post("/users", json={"username": "  "})).status == 400         # empty
        users = (await (await c.get("/users")).json())["users"]
        assert users[uid] == "alice b"
        h = {"comfy-user": uid}
        assert (await c.post("/settings/theme", json="dark", headers=h)).status == 200
        assert await (await c.get("/settings/theme", headers=h)).json() == "dark"
        assert (await c.get("/userdata/x.json", headers={"comfy-user": "mallory"})).status == 403
    _run(env, fn, multi_user=True)
