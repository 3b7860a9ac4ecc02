"""DVD rip & queue (reference rips/dvd_rip_queue.py).

Optical-disc ingest that feeds the transcode cluster through the manager's
``POST /add_job {mark_watcher_processed: true}``:

1. ``makemkvcon --robot info`` -> :func:`parse_makemkv_robot_output` (CINFO/TINFO/SINFO);
2. :func:`choose_main_title` — longest title at least ``min_seconds`` (40 min) long;
3. title detection — hints from the disc label / udev / MakeMKV fields
   (:func:`build_auto_title_hints`), TMDb search + details scored on title similarity,
   runtime agreement and hint-source reliability (:func:`score_candidate`); a low score
   sends the rip to a staging folder for manual review with a JSON manifest;
4. ``makemkvcon mkv`` rip, then a remux keeping the video, the default audio and English
   subtitles (:func:`remux_plan`), named
   ``WATCH_ROOT/movies/<Title (Year)>/<Title (Year)> <H>p <codec>.mkv``;
5. queue with the manager (or simply drop into the watch folder).

External tools (makemkvcon, ffmpeg) and the TMDb API are injected / optional: every
decision function is pure and unit-tested with recorded MakeMKV output.
"""
from __future__ import annotations

import csv
import difflib
import json
import os
import re
import shutil
import subprocess
import sys
import unicodedata
from pathlib import Path
from typing import Any, Callable

TITLE_INFO = {1: "type", 2: "name", 3: "lang_code", 4: "lang_name", 5: "codec_id", 6: "codec_short",
              7: "codec_long", 8: "chapters", 9: "duration", 10: "size_human", 11: "bytes", 12: "extension",
              13: "bitrate", 14: "audio_channels", 15: "angle_info", 16: "source_name", 17: "sample_rate",
              18: "sample_size", 19: "video_size", 20: "aspect_ratio", 21: "frame_rate", 22: "stream_flags",
              23: "date_time", 27: "output_name", 30: "description", 49: "title_name"}
ENGLISH = {"en", "eng"}
YEAR_RE = re.compile(r"\b((?:19|20)\d{2})\b")
FALLBACK_TITLE = "dvd-rip"
GENERIC_HINTS = {"", "disc", "dvd", "dvd video", "video", "movie", "not identified", "unknown", "untitled",
                 "video ts", "ts"}
LOW_INFO_RE = re.compile(r"^[a-z]{1,3}\d{1,3}[a-z]{0,2}$", re.IGNORECASE)
SOURCE_BONUS = {"disc-label": 18.0, "device-label": 12.0, "disc-info": 4.0, "title-source_name": -2.0,
                "title-output_name": -12.0, "title-title_name": -8.0, "title-name": -8.0}
_NOISE = (r"\b16x9\b", r"\bws\b", r"\bfullscreen\b", r"\bwidescreen\b", r"\bspecial edition\b",
          r"\bcollector'?s edition\b", r"\btheatrical\b", r"\bunrated\b", r"\bblu[- ]?ray\b", r"\bdvd\b",
          r"\bdisc\s*\d+\b", r"\bside\s*[ab12]\b", r"\bsku\b")


# ------------------------------------------------------------------ parsing
def parse_hms_seconds(value) -> int:
    parts = str(value or "").strip().split(":")
    try:
        nums = [int(p) for p in parts]
    except ValueError:
        return 0
    total = 0
    for n in nums:
        total = total * 60 + n
    return total if len(nums) <= 3 else 0


def _csv(payload: str, n: int):
    try:
        row = next(csv.reader([payload]))
    except (StopIteration, csv.Error):
        return None
    return row if len(row) >= n else None


def parse_makemkv_robot_output(text: str) -> dict:
    titles: dict[int, dict] = {}
    disc: dict[str, str] = {}
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("CINFO:"):
            f = _csv(line[6:], 3)
            if f:
                disc[str(int(f[0]))] = f[2]
        elif line.startswith("TINFO:"):
            f = _csv(line[6:], 4)
            if f:
                t = titles.setdefault(int(f[0]), {"index": int(f[0]), "streams": []})
                t[TITLE_INFO.get(int(f[1]), f"field_{f[1]}")] = f[3]
        elif line.startswith("SINFO:"):
            f = _csv(line[6:], 5)
            if f:
                t = titles.setdefault(int(f[0]), {"index": int(f[0]), "streams": []})
                si = int(f[1])
                while len(t["streams"]) <= si:
                    t["streams"].append({"index": len(t["streams"])})
                t["streams"][si][TITLE_INFO.get(int(f[2]), f"field_{f[2]}")] = f[4]
    out = []
    for t in titles.values():
        t["duration_seconds"] = parse_hms_seconds(t.get("duration"))
        t["size_bytes"] = int(t.get("bytes") or 0) if str(t.get("bytes") or "0").isdigit() else 0
        t["chapters_count"] = int(t.get("chapters") or 0) if str(t.get("chapters") or "0").isdigit() else 0
        out.append(t)
    out.sort(key=lambda t: (t["duration_seconds"], t["size_bytes"], t["chapters_count"], -t["index"]), reverse=True)
    return {"disc_info": disc, "titles": out}


def choose_main_title(parsed: dict, min_seconds: int = 2400) -> dict:
    cands = [t for t in parsed.get("titles", []) if t.get("duration_seconds", 0) >= min_seconds]
    cands = cands or list(parsed.get("titles", []))
    if not cands:
        raise RuntimeError("MakeMKV did not return any titles for this disc.")
    return cands[0]


# -------------------------------------------------------------- title hints
def normalize_title(v: str) -> str:
    v = unicodedata.normalize("NFKD", str(v or "")).encode("ascii", "ignore").decode("ascii").lower()
    v = v.replace("&", " and ")
    v = re.sub(r"[^a-z0-9]+", " ", v)
    return re.sub(r"\s+", " ", v).strip()


def cleanup_title_hint(v: str) -> str:
    c = unicodedata.normalize("NFKD", str(v or "")).encode("ascii", "ignore").decode("ascii")
    c = c.replace("_", " ").replace(".", " ")
    for p in _NOISE:
        c = re.sub(p, " ", c, flags=re.IGNORECASE)
    c = re.sub(r"[\[\](){}]", " ", c)
    c = re.sub(r"\s*-\s*", " - ", c)
    return re.sub(r"\s+", " ", c).strip(" -_")


def split_title_year_hint(v: str) -> tuple[str, str | None]:
    c = cleanup_title_hint(v)
    if not c:
        return "", None
    m = YEAR_RE.search(c)
    title = re.sub(r"\s+", " ", YEAR_RE.sub(" ", c)).strip(" -_") or c
    return title, (m.group(1) if m else None)


def is_generic_hint(v: str) -> bool:
    n = normalize_title(cleanup_title_hint(v))
    return n in GENERIC_HINTS or len(n) < 2


def is_low_information_hint(v: str) -> bool:
    n = normalize_title(cleanup_title_hint(v))
    if not n:
        return True
    words = n.split()
    return len(words) == 1 and bool(LOW_INFO_RE.fullmatch(re.sub(r"[^a-z0-9]", "", words[0])))


def build_auto_title_hints(parsed: dict, title: dict, disc_label: str = "", device_label: str = "") -> list[dict]:
    raw = []
    if disc_label:
        raw.append(("disc-label", disc_label))
    if device_label:
        raw.append(("device-label", device_label))
    for k in ("source_name", "output_name", "title_name", "name"):
        v = str(title.get(k) or "").strip()
        if v:
            raw.append((f"title-{k}", v))
    for v in (parsed.get("disc_info") or {}).values():
        if str(v or "").strip():
            raw.append(("disc-info", str(v).strip()))
    hints, seen = [], set()
    for src, val in raw:
        q, year = split_title_year_hint(val)
        if not q or is_generic_hint(q) or is_low_information_hint(q):
            continue
        key = normalize_title(q)
        if key in seen:
            continue
        seen.add(key)
        hints.append({"query": q, "year_hint": year, "source": src, "raw_value": val})
    return hints


# ------------------------------------------------------------------ scoring
def title_similarity(query_norm: str, candidate_title: str, runtime_seconds: int | None) -> float:
    cand = normalize_title(candidate_title)
    qw = query_norm.split()
    if runtime_seconds and len(qw) == 1 and qw[0] in cand.split():
        return 0.76  # one-word labels ("FELLOWSHIP") should not beat a better runtime match
    return difflib.SequenceMatcher(None, query_norm, cand).ratio()


def runtime_adjustment(runtime_seconds: int | None, candidate_minutes) -> float:
    if not runtime_seconds or not candidate_minutes:
        return 0.0
    delta = abs(int(candidate_minutes) * 60 - runtime_seconds) / 60.0
    return max(-90.0, 25.0 - delta)


def score_candidate(query: str, cand: dict, runtime_seconds: int | None, source: str = "",
                    year_hint: str | None = None) -> float:
    qn = normalize_title(query)
    sim = max(title_similarity(qn, cand.get("title") or "", runtime_seconds),
              title_similarity(qn, cand.get("original_title") or "", runtime_seconds))
    s = sim * 100.0 + runtime_adjustment(runtime_seconds, cand.get("runtime"))
    if cand.get("release_date"):
        s += 1.0
        if year_hint and str(cand["release_date"])[:4] == year_hint:
            s += 10.0
    return round(s + SOURCE_BONUS.get(source, 0.0), 2)


class Tmdb:
    """Minimal TMDb v3 client (search + details); `fetch` is injectable for tests."""

    def __init__(self, api_key: str, fetch: Callable[[str, dict], dict | None] | None = None):
        self.api_key = api_key
        self.fetch = fetch or self._http

    def _http(self, path: str, params: dict) -> dict | None:
        import requests

        try:
            r = requests.get(f"https://api.themoviedb.org/3{path}", params={**params, "api_key": self.api_key},
                             timeout=15)
            return r.json() if r.ok else None
        except (requests.RequestException, ValueError):
            return None

    def search(self, query: str, year: str | None = None) -> list[dict]:
        p = {"query": query, "include_adult": "false"}
        if year:
            p["year"] = year
        return list((self.fetch("/search/movie", p) or {}).get("results") or [])[:8]

    def details(self, movie_id: int) -> dict:
        return self.fetch(f"/movie/{movie_id}", {}) or {}


def auto_detect_movie_metadata(parsed: dict, title: dict, disc_label: str = "", device_label: str = "",
                               tmdb: Tmdb | None = None, min_score: float = 70.0) -> dict:
    runtime = int(title.get("duration_seconds") or 0) or None
    hints = build_auto_title_hints(parsed, title, disc_label, device_label)
    if not hints:
        return {"title": FALLBACK_TITLE, "year": None, "source": "auto-title-unavailable",
                "needs_manual_review": True, "review_reason": "no usable title hints in the disc metadata"}
    best = None
    if tmdb is not None:
        for h in hints:
            for c in tmdb.search(h["query"], h["year_hint"]):
                d = {**c, **tmdb.details(c["id"])} if c.get("id") is not None else c
                sc = score_candidate(h["query"], d, runtime, h["source"], h["year_hint"])
                if best is None or sc > best[0]:
                    best = (sc, d, h)
    if best is None:
        h = hints[0]
        return {"title": h["query"].title(), "year": h["year_hint"], "source": h["source"], "score": None,
                "needs_manual_review": True, "review_reason": "no TMDb match (offline or no API key)"}
    sc, d, h = best
    year = str(d.get("release_date") or "")[:4] or h["year_hint"]
    out = {"title": d.get("title") or h["query"], "year": year, "tmdb_id": d.get("id"), "score": sc,
           "source": h["source"], "query_used": h["query"], "needs_manual_review": sc < min_score}
    if out["needs_manual_review"]:
        out["review_reason"] = f"best TMDb score {sc:.1f} < {min_score:.1f}"
    return out


# ------------------------------------------------------------- naming / streams
def safe_filename(title: str) -> str:
    t = re.sub(r'[<>:"/\\|?*\x00-\x1f]', " ", str(title or ""))
    return re.sub(r"\s+", " ", t).strip(" .") or FALLBACK_TITLE


def display_name(title: str, year: str | None) -> str:
    return f"{safe_filename(title)} ({year})" if year else safe_filename(title)


def unique_path(p: Path) -> Path:
    if not p.exists():
        return p
    for i in range(2, 1000):
        q = p.with_name(f"{p.stem} [{i}]{p.suffix}")
        if not q.exists():
            return q
    raise RuntimeError(f"no free name for {p}")


def build_final_path(watch_root: Path, title: str, year: str | None, height: int, codec: str = "h264",
                     subdir: str = "movies", suffix: str = ".mkv") -> Path:
    name = display_name(title, year)
    return unique_path(Path(watch_root) / subdir / name / f"{name} {int(height)}p {codec}{suffix}")


def stream_language(stream: dict) -> str:
    """ffprobe tags.language, else MakeMKV's lang_code / lang_name."""
    for v in ((stream.get("tags") or {}).get("language"), stream.get("language"), stream.get("lang_code"),
              stream.get("lang_name")):
        if str(v or "").strip():
            return str(v).strip().lower()
    return ""


def is_english(stream: dict) -> bool:
    lang = stream_language(stream)
    return lang in ENGLISH or lang == "english"


def canonical_stream_type(stream: dict) -> str:
    """"video" / "audio" / "subtitle" from ffprobe codec_type or MakeMKV's type field
    ("Video", "Audio", "Subtitles")."""
    k = str(stream.get("codec_type") or stream.get("type") or "").strip().lower()
    return "video" if k.startswith("video") else "audio" if k.startswith("audio") else \
        "subtitle" if k.startswith("sub") else k


def stream_codec(stream: dict) -> str:
    return str(stream.get("codec_name") or stream.get("codec_short") or stream.get("codec_long") or "").strip().lower()


def choose_default_audio(audio: list[dict]) -> dict | None:
    """English AC-3 first (the DVD main mix), then any English track, then the first."""
    return (next((s for s in audio if is_english(s) and stream_codec(s) == "ac3"), None)
            or next((s for s in audio if is_english(s)), None) or (audio[0] if audio else None))


def choose_default_subtitle(subs: list[dict]) -> dict | None:
    return next((s for s in subs if is_english(s)), None)


def remux_plan(streams: list[dict]) -> dict:
    """Stream selection for the remux: all video, the default audio, every English
    subtitle."""
    by = lambda k: [s for s in streams if canonical_stream_type(s) == k]
    a = choose_default_audio(by("audio"))
    return {"video": [s["index"] for s in by("video")], "audio": [a["index"]] if a else [],
            "subtitles": [s["index"] for s in by("subtitle") if is_english(s)]}


def stage_for_manual_review(mkv: Path, staging: Path, meta: dict) -> Path:
    """Move a low-confidence rip into a new staging bundle (see :mod:`.bundle`)."""
    from .bundle import stage

    return stage(mkv, meta, staging, str(meta.get("disc_label") or ""), str(meta.get("title") or "")).mkv


# ------------------------------------------------------------- configuration
def load_env_file(path) -> dict:
    """KEY=value lines of a shell-style defaults file (``export`` and quotes allowed)."""
    import shlex

    p = Path(path).expanduser()
    if not p.is_file():
        return {}
    out = {}
    for line in p.read_text(encoding="utf-8").splitlines():
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        if line.startswith("export "):
            line = line[7:].strip()
        m = re.match(r"^([A-Za-z_][A-Za-z0-9_]*)=(.*)$", line)
        if not m:
            continue
        try:
            v = " ".join(shlex.split(m.group(2))) if m.group(2).strip() else ""
        except ValueError:
            v = m.group(2).strip()
        out[m.group(1)] = v
    return out


def configured(file_cfg: dict, *names: str, fallback=None, cast=str):
    """First non-empty of the environment variables `names`, then the defaults file's
    entry for names[0], else `fallback` (also when the value does not parse)."""
    for v in [os.environ.get(n) for n in names] + [file_cfg.get(names[0])]:
        if v not in (None, ""):
            try:
                return cast(v)
            except ValueError:
                return fallback
    return fallback


def submit_add_job(manager_url: str, rel_filename: str, input_path: str | None = None, post=None) -> dict:
    import requests

    payload = {"filename": rel_filename, "mark_watcher_processed": True}
    if input_path:
        payload["input_path"] = input_path
    url = manager_url.rstrip("/")
    url = url if url.endswith("/add_job") else url + "/add_job"
    r = (post or requests.post)(url, json=payload, timeout=20)
    return r.json()


# ---------------------------------------------------------------------- CLI
def main(argv=None) -> int:  # pragma: no cover - thin wrapper, see cli.run
    from .cli import main as _main

    return _main(argv)
