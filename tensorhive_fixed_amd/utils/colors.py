"""ANSI colour helpers for CLI and terminal warnings."""


def red(s: str) -> str:
    return f"\033[91m{s}\033[0m"


def green(s: str) -> str:
    return f"\033[92m{s}\033[0m"


def orange(s: str) -> str:
    return f"\033[93m{s}\033[0m"


def bold(s: str) -> str:
    return f"\033[1m{s}\033[0m"
