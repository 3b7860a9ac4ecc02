"""Interactive title / stream selection for ``--select-streams`` (reference
rips/dvd_rip_queue.py prompt_for_title_selection :747-777, parse_menu_selection :1438-1471,
prompt_for_stream_selection :1474-1586).

Menus are 1-based; Enter keeps the automatic pick.  The picks are returned as
(codec_type, ordinal within that type) because MakeMKV's stream numbering differs from the
ripped MKV's — :func:`tools.resolve_selection` maps them after the rip.  `ask` and `out` are
injectable so the prompts are testable without a terminal.
"""
from __future__ import annotations

import sys
from typing import Callable

from . import canonical_stream_type, choose_default_audio, choose_default_subtitle


def _tty() -> bool:
    return sys.stdin.isatty()


def title_label(t: dict) -> str:
    parts = [f"title={t.get('index', '?')}"]
    if t.get("duration"):
        parts.append(str(t["duration"]))
    if t.get("chapters_count"):
        parts.append(f"chapters={t['chapters_count']}")
    if int(t.get("size_bytes") or 0) > 0:
        parts.append(f"size={int(t['size_bytes']) / 2 ** 30:.2f}GiB")
    name = t.get("source_name") or t.get("output_name") or t.get("title_name") or ""
    if name:
        parts.append(str(name))
    return " | ".join(parts)


def stream_label(s: dict) -> str:
    tags = s.get("tags") or {}
    kind = canonical_stream_type(s)
    parts = [f"stream={s.get('index', '?')}", kind]
    codec = s.get("codec_name") or s.get("codec_short") or s.get("codec_long") or ""
    if codec:
        parts.append(str(codec).lower())
    if kind == "video":
        size = f"{s['width']}x{s['height']}" if s.get("width") and s.get("height") else s.get("video_size") or ""
        if size:
            parts.append(size)
    elif kind == "audio":
        ch = s.get("channels") or s.get("audio_channels")
        if ch:
            parts.append(f"{ch}ch")
        if s.get("channel_layout"):
            parts.append(s["channel_layout"])
    lang = tags.get("language") or s.get("lang_code") or s.get("lang_name") or ""
    if lang:
        parts.append(f"lang={lang}")
    name = tags.get("title") or s.get("name") or ""
    if name:
        parts.append(f"title={name}")
    return " | ".join(p for p in parts if p)


def parse_menu(raw: str, items: list, multiple: bool = False, allow_none: bool = False) -> list | None:
    """1-based picks ("2", "1,3", "none") -> items; None when the answer is invalid or
    empty (the caller applies the default)."""
    raw = raw.strip().lower()
    if raw == "none" and allow_none:
        return []
    pieces = [p.strip() for p in raw.split(",") if p.strip()]
    if not pieces or (not multiple and len(pieces) != 1):
        return None
    out, seen = [], set()
    for p in pieces:
        if not p.isdigit() or not 1 <= int(p) <= len(items):
            return None
        if int(p) not in seen:
            seen.add(int(p))
            out.append(items[int(p) - 1])
    return out


def _choose(items: list, label: Callable, what: str, default, ask, out, allow_none: bool = False):
    out(f"Select {what}:")
    for i, it in enumerate(items, 1):
        out(f"  {i}. {label(it)}")
    dflt = f"{items.index(default) + 1}" if default is not None else "none"
    if default is not None:
        out(f"Auto-selected {what}: {dflt} ({label(default)})")
    while True:
        raw = ask(f"Choose one {what} [{dflt}]{' (or none)' if allow_none else ''}: ")
        if not raw.strip():
            return default
        pick = parse_menu(raw, items, allow_none=allow_none)
        if pick is not None:
            return pick[0] if pick else None
        out(f"Enter one number from the {what} list{' or none' if allow_none else ''}.")


def choose_title(parsed: dict, default: dict, ask=input, out=None, tty=_tty) -> dict:
    if not tty():
        raise RuntimeError("interactive title selection needs a terminal")
    titles = list(parsed.get("titles") or [])
    if not titles:
        raise RuntimeError("MakeMKV did not return any titles for this disc")
    return _choose(titles, title_label, "title", default, ask, out or (lambda m: print(m, file=sys.stderr)))


def choose_streams(streams: list[dict], ask=input, out=None, tty=_tty) -> list[dict]:
    """One video, one audio (default English AC-3 / English / first) and at most one
    subtitle (default first English, or none) -> [{codec_type, ordinal}]."""
    if not tty():
        raise RuntimeError("interactive stream selection needs a terminal")
    out = out or (lambda m: print(m, file=sys.stderr))
    by = {k: [s for s in streams if canonical_stream_type(s) == k] for k in ("video", "audio", "subtitle")}
    if not by["video"]:
        raise RuntimeError("the selected title has no video stream")
    picks = [_choose(by["video"], stream_label, "video stream", by["video"][0], ask, out)]
    if by["audio"]:
        picks.append(_choose(by["audio"], stream_label, "audio stream", choose_default_audio(by["audio"]), ask, out))
    if by["subtitle"]:
        picks.append(_choose(by["subtitle"], stream_label, "subtitle stream", choose_default_subtitle(by["subtitle"]),
                             ask, out, allow_none=True))
    res = []
    for s in picks:
        if s is None:
            continue
        k = canonical_stream_type(s)
        res.append({"codec_type": k, "ordinal": by[k].index(s)})
    return res
