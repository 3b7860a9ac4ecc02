"""External-tool layer of the rip tool: makemkvcon (robot mode), ffprobe, ffmpeg, blkid /
udevadm.  Every call goes through a :class:`Runner` so tests substitute recorded output
(reference: rips/dvd_rip_queue.py run_command :205-246, stream_makemkv_command :256-334,
resolve_source_spec :552-575, probe_disc_label :578-600, ffprobe_streams :1238-1256,
remux_with_english_subtitles :1616-1676).

MakeMKV robot progress (``--progress=-same``) arrives as PRGT (task title), PRGC (current
action) and PRGV (current, total, max) lines; :class:`ProgressFilter` turns that stream into
a few human lines (every 5 % overall / 10 % current step), so a 30-minute rip prints ~20
lines instead of thousands.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
from dataclasses import dataclass, field
from pathlib import Path
from typing import Callable, Iterable

from . import _csv, canonical_stream_type, choose_default_audio, choose_default_subtitle, is_english


@dataclass
class Result:
    returncode: int
    stdout: str = ""
    stderr: str = ""


class Runner:
    """Runs external commands.  ``lines(cmd)`` yields merged stdout/stderr lines as they are
    produced (for progress streaming), ``run(cmd)`` captures.  ``which`` answers tool
    availability.  Subclass / replace in tests."""

    def which(self, name: str) -> bool:
        return shutil.which(name) is not None

    def run(self, cmd: list[str]) -> Result:
        p = subprocess.run(cmd, capture_output=True, text=True)
        return Result(p.returncode, p.stdout, p.stderr)

    def lines(self, cmd: list[str]) -> tuple[Iterable[str], Callable[[], int]]:
        p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, bufsize=1)
        return (p.stdout if p.stdout is not None else iter(())), p.wait


def say(msg: str) -> None:
    print(msg, file=sys.stderr, flush=True)


@dataclass
class ProgressFilter:
    prefix: str
    sink: Callable[[str], None] = say
    task: str = ""
    action: str = ""
    last: tuple | None = None
    shown: list = field(default_factory=list)

    def feed(self, line: str) -> None:
        line = line.strip()
        kind, _, payload = line.partition(":")
        if kind in ("PRGT", "PRGC"):
            f = _csv(payload, 3)
            label = (f[-1] if f else payload).strip()
            if kind == "PRGT":
                self.task = label
            else:
                if label == self.task:
                    return
                self.action = label
            if label:
                self._emit(f"{self.prefix}: {label}")
        elif kind == "PRGV":
            f = _csv(payload, 3)
            try:
                cur, tot, mx = (int(x) for x in f[:3]) if f else (0, 0, 0)
            except ValueError:
                return
            if mx <= 0:
                return
            tp = max(0, min(100, round(100 * tot / mx)))
            cp = max(0, min(100, round(100 * cur / mx)))
            label = self.action or self.task or "working"
            mark = (label, tp // 5, cp // 10)
            if mark == self.last:
                return
            self.last = mark
            self._emit(f"{self.prefix}: {label} ({tp}%)" if tp == cp else
                       f"{self.prefix}: {label} ({tp}% overall, {cp}% current)")

    def _emit(self, msg: str) -> None:
        self.shown.append(msg)
        self.sink(msg)


def stream_makemkv(runner: Runner, cmd: list[str], prefix: str, sink=say, debug: bool = False) -> Result:
    """Run makemkvcon, reporting progress as it goes; returns the full output."""
    it, wait = runner.lines(cmd)
    pf = ProgressFilter(prefix, sink)
    out = []
    for raw in it:
        out.append(raw if raw.endswith("\n") else raw + "\n")
        if debug and raw.strip():
            sink(f"[makemkv] {raw.rstrip()}")
        pf.feed(raw)
    return Result(wait(), "".join(out))


def parse_drive_scan(text: str) -> list[dict]:
    """DRV:index,visible,enabled,flags,drive name,disc name,device path lines."""
    drives = []
    for line in text.splitlines():
        line = line.strip()
        if not line.startswith("DRV:"):
            continue
        f = _csv(line[4:], 7)
        if not f or not f[0].strip().lstrip("-").isdigit():
            continue
        drives.append({"index": int(f[0]), "visible": f[1], "enabled": f[2], "flags": f[3], "drive_name": f[4],
                       "disc_name": f[5], "device_path": f[6]})
    return drives


def resolve_source(runner: Runner, source: str, device: str) -> str:
    """MakeMKV source spec: explicit, or ``auto`` = the disc:N whose drive is `device`."""
    if source and source != "auto":
        return source
    want = os.path.realpath(os.path.expanduser(device))
    r = runner.run(["makemkvcon", "--robot", "info", "disc:9999"])
    if r.returncode == 0:
        for d in parse_drive_scan(r.stdout):
            p = (d["device_path"] or "").strip()
            if p and os.path.realpath(p) == want:
                return f"disc:{d['index']}"
    return "disc:0"


def probe_disc_label(runner: Runner, device: str) -> str:
    dev = os.path.expanduser(device)
    if runner.which("blkid"):
        r = runner.run(["blkid", "-o", "value", "-s", "LABEL", dev])
        if r.returncode == 0 and r.stdout.strip():
            return r.stdout.strip()
    if runner.which("udevadm"):
        r = runner.run(["udevadm", "info", "--query=property", "--name", dev])
        if r.returncode == 0:
            for line in r.stdout.splitlines():
                if line.startswith("ID_FS_LABEL="):
                    return line.split("=", 1)[1].strip()
    return ""


def ffprobe_streams(runner: Runner, path: Path) -> list[dict]:
    r = runner.run(["ffprobe", "-v", "error", "-show_entries",
                    "stream=index,codec_type,codec_name,width,height,channels,channel_layout:stream_tags=language,title",
                    "-of", "json", str(path)])
    if r.returncode != 0:
        raise RuntimeError(f"ffprobe failed on {path}: {r.stderr.strip()[:500]}")
    return list((json.loads(r.stdout or "{}") or {}).get("streams") or [])


def resolution_label(runner: Runner, path: Path) -> str:
    if not runner.which("ffprobe"):
        return "unknown"
    for s in ffprobe_streams(runner, path):
        try:
            if s.get("codec_type") == "video" and int(s.get("height") or 0) > 0:
                return f"{int(s['height'])}p"
        except (TypeError, ValueError):
            continue
    return "unknown"


def resolve_selection(runner: Runner, specs: list[dict], mkv: Path) -> list[dict]:
    """Map (type, ordinal) picks made on MakeMKV's title streams onto the ripped file's
    ffprobe streams (MakeMKV and ffprobe number streams differently; per-type order agrees)."""
    streams = ffprobe_streams(runner, mkv)
    out = []
    for sp in specs:
        of_type = [s for s in streams if canonical_stream_type(s) == sp["codec_type"]]
        if not 0 <= int(sp["ordinal"]) < len(of_type):
            raise RuntimeError(f"selected {sp['codec_type']} stream #{int(sp['ordinal']) + 1} is not in the ripped MKV")
        out.append(of_type[int(sp["ordinal"])])
    return out


def remux(runner: Runner, src: Path, dst: Path, title: str, selected: list[dict] | None = None) -> bool | None:
    """Stream-copy remux keeping the chosen streams — by default all video, the default
    audio (English AC-3 first) and the first English subtitle — with chapters and metadata.
    Returns whether English subtitles were kept, or None when ffmpeg/ffprobe are missing
    (the raw rip is used as is)."""
    if not (runner.which("ffmpeg") and runner.which("ffprobe")):
        return None
    if selected is None:
        streams = ffprobe_streams(runner, src)
        a = choose_default_audio([s for s in streams if canonical_stream_type(s) == "audio"])
        sub = choose_default_subtitle([s for s in streams if canonical_stream_type(s) == "subtitle"])
        maps = ["-map", "0:v"] + (["-map", f"0:{int(a['index'])}"] if a else []) + \
               (["-map", f"0:{int(sub['index'])}"] if sub else [])
        kept = sub is not None
    else:
        maps = [x for s in selected for x in ("-map", f"0:{int(s['index'])}")]
        kept = any(canonical_stream_type(s) == "subtitle" and is_english(s) for s in selected)
    r = runner.run(["ffmpeg", "-hide_banner", "-nostats", "-loglevel", "error", "-y", "-i", str(src), *maps,
                    "-map_metadata", "0", "-map_chapters", "0", "-metadata", f"title={title}", "-c", "copy", str(dst)])
    if r.returncode != 0:
        raise RuntimeError(f"ffmpeg remux failed: {r.stderr.strip()[:1000]}")
    return kept


def find_single_mkv(path: Path) -> Path:
    mkvs = sorted(p for p in path.rglob("*.mkv") if p.is_file())
    if len(mkvs) != 1:
        raise RuntimeError(f"expected exactly one MKV under {path}, found {len(mkvs)}: {[str(m) for m in mkvs]}")
    return mkvs[0]
