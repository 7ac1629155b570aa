"""Users & settings (parity: ``app/user_manager.py:14-140``, ``app/app_settings.py:6-54``; C03).

``--multi-user`` profiles selected by the ``comfy-user`` header, ``users.json``, per-user
``userdata/{file}`` GET/POST with path-escape guards, ``/settings[/{id}]`` JSON store.
"""
from __future__ import annotations

import json
import os
import re
import uuid

from aiohttp import web

from ..utils import folder_paths


class UserManager:
    def __init__(self, multi_user=False):
        self.multi_user = multi_user
        user_directory = folder_paths.get_user_directory()
        self.users_file = os.path.join(user_directory, "users.json")
        if multi_user and os.path.isfile(self.users_file):
            with open(self.users_file) as f:
                self.users = json.load(f)
        else:
            self.users = {}

    def get_users_file(self):
        return os.path.join(folder_paths.get_user_directory(), "users.json")

    def get_request_user_id(self, request):
        user = "default"
        if self.multi_user and "comfy-user" in request.headers:
            user = request.headers["comfy-user"]
        if user not in self.users and self.multi_user:
            raise KeyError("Unknown user: " + user)
        return user

    def get_request_user_filepath(self, request, file, type="userdata", create_dir=True):
        user_directory = folder_paths.get_user_directory()
        if type == "userdata":
            root_dir = user_directory
        else:
            raise KeyError("Unknown filepath type:" + type)
        user = self.get_request_user_id(request)
        path = user_root = os.path.abspath(os.path.join(root_dir, user))
        if os.path.commonpath((root_dir, user_root)) != os.path.abspath(root_dir):
            return None
        if file is not None:
            path = os.path.abspath(os.path.join(user_root, file))
            if os.path.commonpath((user_root, path)) != user_root:
                return None
        parent = os.path.split(path)[0]
        if create_dir and not os.path.exists(parent):
            os.makedirs(parent, exist_ok=True)
        return path

    def add_user(self, name):
        name = name.strip()
        if not name:
            raise ValueError("username not provided")
        user_id = re.sub("[^a-zA-Z0-9-_]+", "-", name)
        user_id = user_id + "_" + str(uuid.uuid4())
        self.users[user_id] = name
        os.makedirs(os.path.dirname(self.get_users_file()), exist_ok=True)
        with open(self.get_users_file(), "w") as f:
            json.dump(self.users, f)
        return user_id

    def add_routes(self, routes):
        @routes.get("/users")
        async def get_users(request):
            if self.multi_user:
                return web.json_response({"storage": "server", "users": self.users})
            user_dir = self.get_request_user_filepath(request, None, create_dir=False)
            return web.json_response({"storage": "server", "migrated": os.path.exists(user_dir)})

        @routes.post("/users")
        async def post_users(request):
            body = await request.json()
            username = body.get("username", "")
            if username in self.users.values():
                return web.json_response({"error": "Duplicate username."}, status=400)
            try:
                user_id = self.add_user(username)
            except ValueError as e:
                return web.json_response({"error": str(e)}, status=400)
            return web.json_response(user_id)

        @routes.get("/userdata/{file}")
        async def getuserdata(request):
            file = request.match_info.get("file", None)
            if not file:
                return web.Response(status=400)
            try:
                path = self.get_request_user_filepath(request, file)
            except KeyError:
                return web.Response(status=403)
            if not path:
                return web.Response(status=403)
            if not os.path.exists(path):
                return web.Response(status=404)
            return web.FileResponse(path)

        @routes.post("/userdata/{file}")
        async def post_userdata(request):
            file = request.match_info.get("file", None)
            if not file:
                return web.Response(status=400)
            try:
                path = self.get_request_user_filepath(request, file)
            except KeyError:
                return web.Response(status=403)
            if not path:
                return web.Response(status=403)
            overwrite = request.query.get("overwrite", "true") != "false"
            if not overwrite and os.path.exists(path):
                return web.Response(status=409)
            body = await request.read()
            with open(path, "wb") as f:
                f.write(body)
            return web.Response(status=200)


class AppSettings:
    def __init__(self, user_manager):
        self.user_manager = user_manager

    def get_settings(self, request):
        file = self.user_manager.get_request_user_filepath(request, "comfy.settings.json")
        if os.path.isfile(file):
            with open(file) as f:
                return json.load(f)
        return {}

    def save_settings(self, request, settings):
        file = self.user_manager.get_request_user_filepath(request, "comfy.settings.json")
        with open(file, "w") as f:
            f.write(json.dumps(settings, indent=4))

    def add_routes(self, routes):
        @routes.get("/settings")
        async def get_settings(request):
            return web.json_response(self.get_settings(request))

        @routes.get("/settings/{id}")
        async def get_setting(request):
            value = None
            settings = self.get_settings(request)
            setting_id = request.match_info.get("id", None)
            if setting_id and setting_id in settings:
                value = settings[setting_id]
            return web.json_response(value)

        @routes.post("/settings")
        async def post_settings(request):
            settings = self.get_settings(request)
            new_settings = await request.json()
            self.save_settings(request, {**settings, **new_settings})
            return web.Response(status=200)

        @routes.post("/settings/{id}")
        async def post_setting(request):
            setting_id = request.match_info.get("id", None)
            if not setting_id:
                return web.Response(status=400)
            settings = self.get_settings(request)
            settings[setting_id] = await request.json()
            self.save_settings(request, settings)
            return web.Response(status=200)
