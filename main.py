"""`python main.py [flags]` — same entry point as the reference (see comfy_gen_server_amd/main.py)."""
from comfy_gen_server_amd.main import main

if __name__ == "__main__":
    raise SystemExit(main())
