"""Progress bar with a global hook (parity: ``comfy/utils.py:456-483``): the server installs a hook
that turns every update into a WS ``progress`` event (+ binary preview frame) and checks the
interrupt flag (``main.py:152-160``)."""
from __future__ import annotations

PROGRESS_BAR_ENABLED = True
PROGRESS_BAR_HOOK = None


def set_progress_bar_enabled(enabled):
    global PROGRESS_BAR_ENABLED
    PROGRESS_BAR_ENABLED = enabled


def set_progress_bar_global_hook(function):
    global PROGRESS_BAR_HOOK
    PROGRESS_BAR_HOOK = function


class ProgressBar:
    def __init__(self, total):
        self.total = total
        self.current = 0
        self.hook = PROGRESS_BAR_HOOK

    def update_absolute(self, value, total=None, preview=None):
        if total is not None:
            self.total = total
        if value > self.total:
            value = self.total
        self.current = value
        if self.hook is not None:
            self.hook(self.current, self.total, preview)

    def update(self, value):
        self.update_absolute(self.current + value)
