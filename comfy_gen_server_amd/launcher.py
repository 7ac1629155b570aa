"""Launcher: build the web client if stale, then run the engine locally or serve the UI against a
remote engine (C04; the reference's ``start.py:1-149`` + ``static_file_server.py``).

    python -m comfy_gen_server_amd.launcher [--mode local|remote] [--remote-url URL] [--no-browser]
                                            [-- <engine args>]

* The client build (``web/``, any of yarn / npm / pnpm) is re-run only when a file under ``web/src``
  is newer than ``web/dist`` (the reference's ``is_build_up_to_date``); with no package manager or no
  sources the launcher serves whatever is there.
* ``local``: the engine (``python -m comfy_gen_server_amd.main``) runs as a CHILD process -- it
  initialises the GPUs, this process never does -- and its exit code is passed through.
* ``remote``: a small aiohttp server hosts the built client and answers ``/launcher/config.json``
  with the remote API base and transport (``grpc``), so the client talks to a remote gen-server.
  The access token comes from ``CGS_REMOTE_TOKEN`` or a per-user token file (mode 0600; the
  reference keeps it in the OS keyring, not installed here); without one, the login flow of the
  reference runs: a one-shot callback server on ``--login-port`` receives ``?token=`` from the
  login page and stores it.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import shutil
import subprocess
import sys
import webbrowser

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WEB_DIR = os.path.join(ROOT, "web")
TOKEN_FILE = os.path.join(os.path.expanduser("~"), ".config", "comfy_gen_server_amd", "token")


def _latest_mtime(path: str) -> float:
    latest = os.path.getmtime(path)
    for root, dirs, files in os.walk(path):
        for name in dirs + files:
            try:
                latest = max(latest, os.path.getmtime(os.path.join(root, name)))
            except OSError:
                pass
    return latest


def build_up_to_date(web_dir: str = WEB_DIR) -> bool:
    """True when there is nothing to build: no sources, or ``dist`` newer than every source file."""
    src, dist = os.path.join(web_dir, "src"), os.path.join(web_dir, "dist")
    if not os.path.isdir(src):
        return True
    if not os.path.isdir(dist):
        return False
    return _latest_mtime(src) <= _latest_mtime(dist)


def package_manager():
    for m in ("yarn", "npm", "pnpm"):
        if shutil.which(m):
            return m
    return None


def build_client(web_dir: str = WEB_DIR) -> bool:
    """Install the client's JS dependencies and build it; False when no package manager exists."""
    m = package_manager()
    if m is None:
        print("launcher: no yarn/npm/pnpm found; serving the existing client build", file=sys.stderr)
        return False
    subprocess.run([m, "install"], check=True, cwd=web_dir)
    subprocess.run([m, "build"] if m == "yarn" else [m, "run", "build"], check=True, cwd=web_dir)
    return True


# -- token store (file instead of the OS keyring) ---------------------------------------------------
def load_token(path: str = TOKEN_FILE):
    tok = os.environ.get("CGS_REMOTE_TOKEN")
    if tok:
        return tok
    try:
        with open(path) as f:
            return f.read().strip() or None
    except OSError:
        return None


def store_token(token: str, path: str = TOKEN_FILE):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    with os.fdopen(fd, "w") as f:
        f.write(token)


async def login(login_url: str, port: int, path: str = TOKEN_FILE, open_browser=True) -> str:
    """One-shot callback server: the login page redirects to ``http://localhost:<port>/?token=...``."""
    from aiohttp import web
    got = asyncio.get_running_loop().create_future()

    async def handle(request):
        token = request.rel_url.query.get("token")
        if token and not got.done():
            store_token(token, path)
            got.set_result(token)
        return web.Response(text="Login successful. You can close this window.")

    app = web.Application()
    app.add_routes([web.get("/", handle)])
    runner = web.AppRunner(app)
    await runner.setup()
    await web.TCPSite(runner, "localhost", port).start()
    target = f"{login_url}?redirect_uri=http://localhost:{port}"
    print(f"launcher: log in at {target}", file=sys.stderr)
    if open_browser:
        webbrowser.open(target)
    try:
        return await got
    finally:
        await runner.cleanup()


# -- remote mode: static client + config --------------------------------------------------------------
def remote_app(dist_dir: str, api_base: str, transport: str = "grpc"):
    from aiohttp import web
    app = web.Application()
    cfg = {"api_base": api_base, "transport": transport}

    async def config(_request):
        return web.json_response(cfg)

    async def index(_request):
        idx = os.path.join(dist_dir, "index.html")
        if os.path.exists(idx):
            return web.FileResponse(idx)
        return web.Response(text=f"no client build in {dist_dir}", status=404)

    app.router.add_get("/launcher/config.json", config)
    app.router.add_get("/", index)
    if os.path.isdir(dist_dir):
        app.router.add_static("/", dist_dir, show_index=False)
    return app


async def serve_remote(args):
    from aiohttp import web
    token = load_token()
    if not token:
        token = await login(args.login_url, args.login_port, open_browser=not args.no_browser)
    base = f"{args.remote_url.rstrip('/')}/{token}"
    runner = web.AppRunner(remote_app(os.path.join(WEB_DIR, "dist"), base, "grpc"))
    await runner.setup()
    await web.TCPSite(runner, "localhost", args.port).start()
    print(f"launcher: UI at http://localhost:{args.port} against {args.remote_url}", file=sys.stderr)
    if not args.no_browser:
        webbrowser.open(f"http://localhost:{args.port}")
    await asyncio.Event().wait()


def local_command(engine_args):
    return [sys.executable, "-m", "comfy_gen_server_amd.main"] + list(engine_args)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    engine_args = []
    if "--" in argv:
        i = argv.index("--")
        argv, engine_args = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--mode", choices=["local", "remote"], default=None)
    ap.add_argument("--port", type=int, default=8188)
    ap.add_argument("--remote-url", default=os.environ.get("CGS_REMOTE_URL", "https://api.void.tech"))
    ap.add_argument("--login-url", default=os.environ.get("CGS_LOGIN_URL", "https://void.tech/login"))
    ap.add_argument("--login-port", type=int, default=3003)
    ap.add_argument("--skip-build", action="store_true")
    ap.add_argument("--no-browser", action="store_true")
    args = ap.parse_args(argv)
    if not args.skip_build and not build_up_to_date():
        build_client()
    mode = args.mode
    if mode is None:
        if sys.stdin.isatty():
            ans = input("Use a local or remote server? [local/remote] (local): ").strip().lower()
            mode = "remote" if ans.startswith("r") else "local"
        else:
            mode = "local"
    if mode == "local":
        if "--port" not in engine_args:
            engine_args += ["--port", str(args.port)]
        return subprocess.call(local_command(engine_args), cwd=ROOT)
    try:
        asyncio.run(serve_remote(args))
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
