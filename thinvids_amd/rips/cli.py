"""``python -m thinvids_amd.rips`` — rip a DVD's main feature and hand it to the cluster
(reference rips/dvd_rip_queue.py main :1817-2284, same flags and defaults file).

    probe (makemkvcon info, progress streamed) -> title (auto / --title-index / menu)
      -> movie metadata (manual title, TMDb, or disc-label auto-detect with a score gate)
      -> rip (makemkvcon mkv, progress streamed) -> remux (chosen / default streams)
      -> confident: WATCH_ROOT/<subdir>/<Title (Year)>/<Title (Year)> <H>p h264.mkv + manifest,
                    queued through the watcher (watch mode) or POST /add_job (api mode)
         doubtful:  staging bundle (manifest review_status=pending) for --staged-path later
    --staged-path / --rename-path resume from a bundle without touching the drive.

:func:`run` takes its collaborators (tool runner, TMDb client factory, prompt, HTTP post)
as arguments, so the whole flow is exercised in tests with recorded tool output.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time
from pathlib import Path

from . import (FALLBACK_TITLE, Tmdb, auto_detect_movie_metadata, choose_main_title, configured, display_name,
               load_env_file, parse_makemkv_robot_output, safe_filename, score_candidate, split_title_year_hint,
               submit_add_job)
from . import bundle as B
from . import select as S
from . import tools as T

DEFAULT_ENV_FILE = "/etc/default/thinvids-dvd-auto"


def output_subdir(v: str) -> str:
    c = str(v).replace("\\", "/").strip().strip("/")
    if not c or c == "." or ".." in c.split("/") or os.path.isabs(str(v).strip()):
        raise argparse.ArgumentTypeError("output directory must be a relative path under WATCH_ROOT")
    return c


def build_parser(cfg: dict) -> argparse.ArgumentParser:
    home = Path.home()
    ap = argparse.ArgumentParser(prog="thinvids_amd.rips", description=__doc__.split("\n")[0])
    ap.add_argument("title", nargs="?", help="movie title for the ripped file; omit to auto-detect")
    ap.add_argument("--device", default="/dev/sr0")
    ap.add_argument("--source", default="auto", help='MakeMKV source (disc:N) or "auto" to resolve from --device')
    ap.add_argument("--watch-root", default=configured(cfg, "THINVIDS_DVD_WATCH_ROOT", "WATCH_ROOT", fallback="/watch"))
    ap.add_argument("--queue-mode", choices=("watch", "api"),
                    default=configured(cfg, "THINVIDS_DVD_QUEUE_MODE", fallback="watch"))
    ap.add_argument("--manager-url", default=configured(cfg, "THINVIDS_DVD_MANAGER_URL",
                                                        fallback="http://localhost:5005/add_job"))
    ap.add_argument("--tmdb-api-key", default=configured(cfg, "THINVIDS_DVD_TMDB_API_KEY", "TMDB_API_KEY"))
    ap.add_argument("--disc-label", default="", help="disc label hint (e.g. udev ID_FS_LABEL)")
    ap.add_argument("--auto-title-min-score", type=float,
                    default=configured(cfg, "THINVIDS_DVD_AUTO_TITLE_MIN_SCORE", fallback=60.0, cast=float))
    ap.add_argument("--output-subdir", "--output-dir", type=output_subdir,
                    default=output_subdir(configured(cfg, "THINVIDS_DVD_OUTPUT_SUBDIR", fallback="movies")))
    ap.add_argument("--min-seconds", type=int, default=configured(cfg, "THINVIDS_DVD_MIN_SECONDS", fallback=2400, cast=int))
    ap.add_argument("--title-index", type=int, help="MakeMKV title index instead of the automatic pick")
    ap.add_argument("--scratch-root", default=configured(cfg, "THINVIDS_DVD_SCRATCH_ROOT", "DVD_RIP_SCRATCH_ROOT",
                                                         fallback=str(home / "thinvids-dvd-tmp")))
    ap.add_argument("--staging-root", default=configured(cfg, "THINVIDS_DVD_STAGING_ROOT", "DVD_RIP_STAGING_ROOT",
                                                         fallback=str(home / "thinvids-dvd-staging")))
    ap.add_argument("--staged-path", help="finish a staged rip (bundle dir, manifest or MKV) instead of ripping")
    ap.add_argument("--rename-path", help="rename a finished rip (bundle dir, manifest or MKV) in place")
    ap.add_argument("--select-streams", action="store_true", help="choose title, video, audio and subtitle interactively")
    ap.add_argument("--keep-temp", action="store_true")
    ap.add_argument("--dry-run", action="store_true", help="probe and print the plan without ripping")
    ap.add_argument("--debug", action="store_true", default=configured(cfg, "THINVIDS_DVD_DEBUG", fallback="0") == "1")
    return ap


def validate(a, runner: T.Runner) -> None:
    reuse = bool(a.staged_path or a.rename_path)
    if a.staged_path and a.rename_path:
        raise SystemExit("--staged-path and --rename-path cannot be used together")
    if not reuse and not runner.which("makemkvcon"):
        raise SystemExit("makemkvcon is required but was not found in PATH")
    if a.select_streams and not (runner.which("ffmpeg") and runner.which("ffprobe")):
        raise SystemExit("--select-streams requires ffmpeg and ffprobe")
    if reuse and a.select_streams:
        raise SystemExit("--select-streams cannot be used with --staged-path or --rename-path")
    if reuse and a.title_index is not None:
        raise SystemExit("--title-index cannot be used with --staged-path or --rename-path")
    if reuse and not a.title:
        raise SystemExit("--staged-path and --rename-path need an explicit title to rename the bundle")


def manual_metadata(title: str, tmdb: Tmdb | None, runtime: int | None) -> dict:
    """An explicit title is trusted (no review); TMDb only canonicalises it and adds the
    year when a key is configured."""
    q, year = split_title_year_hint(title)
    q = q or title
    if tmdb is not None:
        best = None
        for c in tmdb.search(q, year):
            d = {**c, **tmdb.details(c["id"])} if c.get("id") is not None else c
            sc = score_candidate(q, d, runtime, "", year)
            if best is None or sc > best[0]:
                best = (sc, d)
        if best is not None:
            sc, d = best
            return {"title": d.get("title") or q, "year": str(d.get("release_date") or "")[:4] or year,
                    "tmdb_id": d.get("id"), "release_date": d.get("release_date"), "score": sc,
                    "source": "manual-input+tmdb", "query_used": q, "needs_manual_review": False}
    return {"title": q, "year": year, "source": "manual-input", "query_used": title, "needs_manual_review": False}


def _diagnostic(scratch: Path, device: str, source: str, out: str) -> Path:
    scratch.mkdir(parents=True, exist_ok=True)
    p = scratch / f"makemkv-info-{Path(device).name or 'device'}-{time.strftime('%Y%m%d-%H%M%S')}.log"
    p.write_text(f"device={device}\nsource={source}\n\n=== output ===\n{out}\n", encoding="utf-8")
    return p


def run(a, runner: T.Runner | None = None, tmdb_factory=Tmdb, ask=input, tty=S._tty, sink=T.say, post=None) -> dict:
    runner = runner or T.Runner()
    validate(a, runner)
    watch, scratch, staging = (Path(x).expanduser() for x in (a.watch_root, a.scratch_root, a.staging_root))
    mode = "staged" if a.staged_path else "rename" if a.rename_path else "new"
    src_bundle: B.Bundle | None = None
    parsed: dict = {"disc_info": {}, "titles": []}
    if mode != "new":
        sink("Loading existing rip bundle...")
        src_bundle = B.locate(a.staged_path or a.rename_path)
        source = str(src_bundle.manifest.get("source") or ("staged-review" if mode == "staged" else "rename-existing"))
        t = src_bundle.manifest.get("selected_title")
        title = t if isinstance(t, dict) else {"index": mode}
    else:
        sink("Resolving MakeMKV source...")
        source = T.resolve_source(runner, a.source, a.device)
        sink("Scanning disc with MakeMKV...")
        probe = T.stream_makemkv(runner, ["makemkvcon", "--robot", "--progress=-same", "info", source], "MakeMKV scan",
                                 sink, a.debug)
        if probe.returncode != 0:
            raise SystemExit(f"makemkvcon info failed (rc {probe.returncode}):\n{probe.stdout[-4000:]}")
        parsed = parse_makemkv_robot_output(probe.stdout)
        if not parsed["titles"]:
            diag = _diagnostic(scratch, a.device, source, probe.stdout)
            raise SystemExit(f"MakeMKV returned no titles; its output is saved in {diag}")
        if a.title_index is not None:
            title = next((t for t in parsed["titles"] if t["index"] == a.title_index), None)
            if title is None:
                raise SystemExit(f"title index {a.title_index} is not on this disc")
        else:
            title = choose_main_title(parsed, a.min_seconds)
            if a.select_streams:
                title = S.choose_title(parsed, title, ask=ask, out=sink, tty=tty)
    runtime = int(title.get("duration_seconds") or 0) or None
    old = src_bundle.manifest if src_bundle else {}
    disc_label = (a.disc_label or old.get("disc_label") or "").strip()
    if not disc_label and mode == "new" and not a.title:
        disc_label = T.probe_disc_label(runner, a.device)
    tmdb = tmdb_factory(a.tmdb_api_key) if a.tmdb_api_key else None
    sink("Resolving movie title...")
    if a.title:
        meta = manual_metadata(a.title, tmdb, runtime)
    else:
        meta = auto_detect_movie_metadata(parsed, title, disc_label, tmdb=tmdb, min_score=a.auto_title_min_score)
    mtitle = str(meta.get("title") or a.title or FALLBACK_TITLE)
    myear = str(meta.get("year") or "") or None
    name = display_name(mtitle, myear)
    sink(f"Using output title: {name}")
    sel_title = {k: title.get(k) for k in ("index", "duration", "duration_seconds", "size_bytes", "chapters_count",
                                           "output_name", "source_name")}
    plan = {"device": a.device, "source": source, "queue_mode": a.queue_mode, "watch_root": str(watch),
            "staged_input": str(src_bundle.mkv) if mode == "staged" else "",
            "rename_input": str(src_bundle.mkv) if mode == "rename" else "",
            "output_path": str(watch / a.output_subdir / name / f"{name} <resolution> h264.mkv"),
            "movie": {k: meta.get(k) for k in ("title", "year", "tmdb_id", "release_date", "source", "query_used")}
            | {"needs_manual_review": bool(meta.get("needs_manual_review")),
               "review_reason": meta.get("review_reason") or ""},
            "selected_title": sel_title}
    if a.dry_run:
        return plan
    picks = S.choose_streams(list(title.get("streams") or []), ask=ask, out=sink, tty=tty) if a.select_streams else None
    tmp_dir = None
    subs_kept = bool(old.get("english_subtitles_kept"))
    staged_out = manifest_path = final = api = None
    try:
        if mode == "new":
            scratch.mkdir(parents=True, exist_ok=True)
            tmp_dir = Path(tempfile.mkdtemp(prefix="thinvids-dvd-", dir=str(scratch)))
            raw = tmp_dir / "raw"
            raw.mkdir()
            sink("Starting rip...")
            r = T.stream_makemkv(runner, ["makemkvcon", "--robot", "--progress=-same", "mkv", source, str(title["index"]),
                                          str(raw)], f"MakeMKV rip title {title['index']}", sink, a.debug)
            if r.returncode != 0:
                raise RuntimeError(f"makemkvcon mkv failed (rc {r.returncode}):\n{r.stdout[-4000:]}")
            raw_mkv = T.find_single_mkv(raw)
            chosen = T.resolve_selection(runner, picks, raw_mkv) if picks is not None else None
            finished = tmp_dir / f"{safe_filename(name)}.mkv"
            kept = T.remux(runner, raw_mkv, finished, mtitle, chosen)
            if kept is None or not finished.exists():
                shutil.move(str(raw_mkv), finished)
                kept = False
            subs_kept = kept
            work = B.Bundle(finished)
        else:
            work = src_bundle
        res = T.resolution_label(runner, work.mkv)
        final = B.unique_dest(watch / a.output_subdir / name / f"{name} {res} h264{work.mkv.suffix or '.mkv'}",
                              current=work.mkv if mode == "rename" else None)
        manifest = {**old, "created_at_epoch": float(old.get("created_at_epoch") or time.time()),
                    "requested_title": a.title or "", "movie_title": meta.get("title"), "movie_year": meta.get("year"),
                    "tmdb_id": meta.get("tmdb_id"), "movie_source": meta.get("source"),
                    "movie_query_used": meta.get("query_used"), "movie_score": meta.get("score"),
                    "needs_manual_review": bool(meta.get("needs_manual_review")),
                    "review_reason": meta.get("review_reason") or "", "disc_label": disc_label,
                    "final_filename": final.name, "device": a.device, "source": source, "selected_title": sel_title,
                    "english_subtitles_kept": bool(subs_kept), "queue_mode": a.queue_mode,
                    "temp_dir": str(tmp_dir) if a.keep_temp and tmp_dir else ""}
        if meta.get("needs_manual_review") and mode != "staged":
            sink("Staging rip for manual review...")
            st = B.stage(work.mkv, manifest, staging, disc_label, name)
            staged_out, manifest_path, final = st.mkv, st.manifest_path, None
        else:
            done = B.finalize(work, final, manifest, mode)
            manifest_path = done.manifest_path
            if a.queue_mode == "api" and mode != "rename":
                api = submit_add_job(a.manager_url, final.relative_to(watch).as_posix(), post=post)
    finally:
        if tmp_dir is not None and not a.keep_temp:
            shutil.rmtree(tmp_dir, ignore_errors=True)
    return {**plan, "english_subtitles_kept": bool(subs_kept),
            "manual_review_required": final is None, "final_path": str(final) if final else "",
            "manifest_path": str(manifest_path) if manifest_path else "",
            "staged_path": str(staged_out) if staged_out else "",
            "rename_path": str(final) if mode == "rename" and final else "",
            "temp_dir": str(tmp_dir) if a.keep_temp and tmp_dir else "", "api_result": api}


def main(argv=None) -> int:  # pragma: no cover - drive + makemkvcon
    cfg = load_env_file(os.environ.get("THINVIDS_DVD_ENV_FILE", DEFAULT_ENV_FILE))
    a = build_parser(cfg).parse_args(argv)
    try:
        out = run(a)
    except (RuntimeError, OSError) as e:
        raise SystemExit(str(e))
    print(json.dumps(out, indent=2, sort_keys=True))
    return 0


if __name__ == "__main__":  # pragma: no cover
    sys.exit(main())
