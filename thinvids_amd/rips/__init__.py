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


def is_english(stream: dict) -> bool:
    return str(stream.get("lang_code") or stream.get("language") or "").strip().lower()[:3] in ENGLISH | {"eng"}


def remux_plan(streams: list[dict]) -> dict:
    """Stream selection for the remux: all video, the default (English-first) audio, every
    English subtitle."""
    kind = lambda s: str(s.get("type") or s.get("codec_type") or "").lower()
    video = [s for s in streams if kind(s).startswith("video")]
    audio = [s for s in streams if kind(s).startswith("audio")]
    subs = [s for s in streams if kind(s).startswith("subtitle")]
    a = next((s for s in audio if is_english(s)), audio[0] if audio else None)
    return {"video": [s["index"] for s in video], "audio": [a["index"]] if a else [],
            "subtitles": [s["index"] for s in subs if is_english(s)]}


def stage_for_manual_review(mkv: Path, staging: Path, meta: dict) -> Path:
    staging.mkdir(parents=True, exist_ok=True)
    dest = unique_path(staging / mkv.name)
    shutil.move(str(mkv), dest)
    with open(dest.with_suffix(".json"), "w") as f:
        json.dump({**meta, "staged_path": str(dest)}, f, indent=2)
    return dest


def submit_add_job(manager_url: str, rel_filename: str, input_path: str | None = None, post=None) -> dict:
    import requests

    payload = {"filename": rel_filename, "mark_watcher_processed": True}
    if input_path:
        payload["input_path"] = input_path
    r = (post or requests.post)(manager_url.rstrip("/") + "/add_job", json=payload, timeout=20)
    return r.json()


# ---------------------------------------------------------------------- CLI
def _run(cmd: list[str], timeout: int = 7200) -> subprocess.CompletedProcess:
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)


def main(argv=None) -> int:  # pragma: no cover - needs a drive + makemkvcon
    import argparse

    ap = argparse.ArgumentParser(description="Rip the main title of a DVD and queue it for transcoding")
    ap.add_argument("--source", default="disc:0")
    ap.add_argument("--watch-root", default=os.environ.get("WATCH_ROOT", "/watch"))
    ap.add_argument("--staging", default=os.environ.get("THINVIDS_DVD_STAGING", "/watch/.staging"))
    ap.add_argument("--manager", default=os.environ.get("THINVIDS_MANAGER_URL", "http://127.0.0.1:5005"))
    ap.add_argument("--disc-label", default="")
    ap.add_argument("--min-seconds", type=int, default=int(os.environ.get("THINVIDS_DVD_MIN_SECONDS", "2400")))
    ap.add_argument("--min-score", type=float, default=float(os.environ.get("THINVIDS_DVD_AUTO_TITLE_MIN_SCORE", "70")))
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args(argv)
    if not shutil.which("makemkvcon"):
        print("makemkvcon not installed", file=sys.stderr)
        return 2
    info = _run(["makemkvcon", "--robot", "--noscan", "info", a.source])
    parsed = parse_makemkv_robot_output(info.stdout)
    title = choose_main_title(parsed, a.min_seconds)
    key = os.environ.get("TMDB_API_KEY")
    meta = auto_detect_movie_metadata(parsed, title, a.disc_label, tmdb=Tmdb(key) if key else None,
                                      min_score=a.min_score)
    print(json.dumps({"title_index": title["index"], "meta": meta}))
    if a.dry_run:
        return 0
    tmp = Path(a.staging) / "rip"
    tmp.mkdir(parents=True, exist_ok=True)
    _run(["makemkvcon", "--robot", "mkv", a.source, str(title["index"]), str(tmp)])
    mkvs = sorted(tmp.glob("*.mkv"))
    if len(mkvs) != 1:
        print(f"expected one MKV, found {len(mkvs)}", file=sys.stderr)
        return 1
    if meta["needs_manual_review"]:
        print("staged for review:", stage_for_manual_review(mkvs[0], Path(a.staging), meta))
        return 0
    height = int(str(title.get("video_size") or "720x480").split("x")[-1] or 480)
    final = build_final_path(Path(a.watch_root), meta["title"], meta.get("year"), height, codec="mpeg2")
    final.parent.mkdir(parents=True, exist_ok=True)
    shutil.move(str(mkvs[0]), final)
    print(json.dumps(submit_add_job(a.manager, str(final.relative_to(a.watch_root)), str(final))))
    return 0
