"""Node-level multi-GPU serving: a rank-0 front end that runs independent prompts on idle ranks and
splits a prompt's image batch across all ranks (SPMD, ``spmd.py``); ``cluster.py`` holds the
coordinator, the worker loop and the rank launcher."""
