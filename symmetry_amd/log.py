"""Console logger with the reference's levels and prefixes (REF ``src/logger.ts``).

Kept quirks: the level enum order DEBUG=0, ERROR=1, INFO=2, WARNING=3 and
default INFO; only ``info`` is gated by the level (``src/logger.ts:28-44``);
``error`` goes to stderr.  Colours are plain ANSI (no chalk), disabled when
the stream is not a TTY or ``NO_COLOR`` is set.
"""
from __future__ import annotations

import enum
import os
import sys


class LogLevel(enum.IntEnum):
    DEBUG = 0
    ERROR = 1
    INFO = 2
    WARNING = 3


_C = {"blue": "\033[34m", "yellow": "\033[33m", "red": "\033[31m", "gray": "\033[90m", "green": "\033[32m",
      "white": "\033[37m", "reset": "\033[0m"}


def _color(stream, name: str, text: str) -> str:
    if os.environ.get("NO_COLOR") or not getattr(stream, "isatty", lambda: False)():
        return text
    return f"{_C[name]}{text}{_C['reset']}"


class Logger:
    _instance: "Logger | None" = None

    def __init__(self):
        self.log_level = LogLevel.INFO
        self.out = sys.stdout
        self.err = sys.stderr

    @classmethod
    def get_instance(cls) -> "Logger":
        if cls._instance is None:
            cls._instance = cls()
        return cls._instance

    def set_log_level(self, level: LogLevel) -> None:
        self.log_level = level

    def _emit(self, stream, prefix: str, color: str, message, args) -> None:
        parts = [_color(stream, color, prefix), str(message)] + [str(a) for a in args]
        print(" ".join(parts), file=stream, flush=True)

    def info(self, message, *args) -> None:
        if self.log_level <= LogLevel.INFO:
            self._emit(self.out, "ℹ️ INFO:", "blue", message, args)

    def warning(self, message, *args) -> None:
        self._emit(self.out, "⚠️ WARNING:", "yellow", message, args)

    def error(self, message, *args) -> None:
        self._emit(self.err, "❌ ERROR:", "red", message, args)

    def debug(self, message, *args) -> None:
        self._emit(self.out, "🐛 DEBUG:", "gray", message, args)


logger = Logger.get_instance()
