"""Launcher (C04, reference start.py) and installer (C61, reference install.py)."""
import asyncio
import os
import sys
import time

import pytest


def test_build_staleness(tmp_path):
    from comfy_gen_server_amd import launcher
    web = tmp_path / "web"
    assert launcher.build_up_to_date(str(web))            # no sources: nothing to build
    (web / "src").mkdir(parents=True)
    (web / "src" / "app.tsx").write_text("x")
    assert not launcher.build_up_to_date(str(web))        # sources, no dist
    (web / "dist").mkdir()
    (web / "dist" / "index.html").write_text("<html/>")
    later = time.time() + 5
    os.utime(web / "dist" / "index.html", (later, later))
    os.utime(web / "dist", (later, later))
    assert launcher.build_up_to_date(str(web))
    newer = later + 5
    os.utime(web / "src" / "app.tsx", (newer, newer))
    assert not launcher.build_up_to_date(str(web))


def test_token_store(tmp_path, monkeypatch):
    from comfy_gen_server_amd import launcher
    monkeypatch.delenv("CGS_REMOTE_TOKEN", raising=False)
    p = str(tmp_path / "cfg" / "token")
    assert launcher.load_token(p) is None
    launcher.store_token("abc123", p)
    assert launcher.load_token(p) == "abc123"
    assert (os.stat(p).st_mode & 0o777) == 0o600
    monkeypatch.setenv("CGS_REMOTE_TOKEN", "envtok")
    assert launcher.load_token(p) == "envtok"


def test_login_callback_and_remote_app(tmp_path):
    from aiohttp import ClientSession
    from aiohttp.test_utils import TestClient, TestServer
    from comfy_gen_server_amd import launcher

    async def run():
        # login: the callback server stores the token the login page redirects with
        p = str(tmp_path / "tok")
        port = 33000 + os.getpid() % 1000
        task = asyncio.ensure_future(launcher.login("https://example.invalid/login", port, p, open_browser=False))
        for _ in range(50):
            await asyncio.sleep(0.05)
            try:
                async with ClientSession() as s:
                    async with s.get(f"http://localhost:{port}/?token=T0K") as r:
                        assert r.status == 200
                break
            except OSError:
                continue
        assert await asyncio.wait_for(task, 10) == "T0K"
        assert launcher.load_token(p) == "T0K"
        # remote mode: client build + config for the remote API
        dist = tmp_path / "dist"
        dist.mkdir()
        (dist / "index.html").write_text("<html>ui</html>")
        (dist / "app.js").write_text("js")
        client = TestClient(TestServer(launcher.remote_app(str(dist), "https://api.example/T0K")))
        await client.start_server()
        try:
            r = await client.get("/launcher/config.json")
            assert (await r.json()) == {"api_base": "https://api.example/T0K", "transport": "grpc"}
            assert "ui" in await (await client.get("/")).text()
            assert (await (await client.get("/app.js")).text()) == "js"
        finally:
            await client.close()
    asyncio.run(run())


def test_local_mode_runs_engine_as_child(monkeypatch):
    from comfy_gen_server_amd import launcher
    calls = []
    monkeypatch.setattr(launcher.subprocess, "call", lambda cmd, cwd=None: calls.append(cmd) or 7)
    rc = launcher.main(["--mode", "local", "--skip-build", "--port", "9001", "--", "--cpu"])
    assert rc == 7
    assert calls[0][:3] == [sys.executable, "-m", "comfy_gen_server_amd.main"]
    assert "--cpu" in calls[0] and calls[0][calls[0].index("--port") + 1] == "9001"


def test_installer_layout_and_checks(tmp_path, capsys):
    from comfy_gen_server_amd import install
    rc = install.main(["--no-build", "--base-directory", str(tmp_path)])
    out = capsys.readouterr().out
    assert "torch" in out and "layout" in out
    for d in ("models/checkpoints", "models/loras", "models/vae", "input", "output", "temp"):
        assert (tmp_path / d).is_dir(), d
    assert install.missing({"os": "os", "definitely_not_a_module_xyz": "nope"}) == ["nope"]
    assert rc in (0, 1)          # 1 only when the CPU container lacks a ROCm GPU stack piece
