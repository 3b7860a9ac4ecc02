"""Rip bundles: an MKV plus its JSON manifest (reference rips/dvd_rip_queue.py :1679-1797).

Low-confidence rips are *staged* — moved into ``<staging root>/<YYYYmmdd-HHMMSS> <label>/``
next to a manifest recording everything the rip decided (disc label, chosen title, TMDb
candidates and score, review reason) with ``review_status = pending``.  Later runs resume
from the bundle instead of re-ripping:

* ``--staged-path X`` — finish a staged rip under a corrected title: the MKV moves into the
  library, its manifest is rewritten next to it (``review_status = resolved``), the staging
  bundle is removed and the job is queued;
* ``--rename-path X`` — rename an already finalised rip in place
  (``review_status = corrected``, ``original_filename`` kept).

X may be the bundle directory, the manifest or the MKV.
"""
from __future__ import annotations

import json
import shutil
import time
from dataclasses import dataclass, field
from pathlib import Path

from . import FALLBACK_TITLE, safe_filename


@dataclass
class Bundle:
    mkv: Path
    manifest_path: Path | None = None
    manifest: dict = field(default_factory=dict)


def write_manifest(path: Path, payload: dict) -> None:
    tmp = path.with_name(path.name + ".tmp")
    tmp.write_text(json.dumps(payload, indent=2, sort_keys=True) + "\n", encoding="utf-8")
    tmp.replace(path)


def read_manifest(path: Path) -> dict:
    d = json.loads(path.read_text(encoding="utf-8"))
    if not isinstance(d, dict):
        raise RuntimeError(f"manifest is not a JSON object: {path}")
    return d


def locate(path) -> Bundle:
    """Bundle from a directory (exactly one .mkv, at most one .json), a manifest (its
    ``staged_mkv`` or sibling .mkv) or an MKV (sibling .json if present)."""
    p = Path(path).expanduser().resolve()
    if not p.exists():
        raise RuntimeError(f"bundle path does not exist: {p}")
    if p.is_dir():
        mkvs = sorted(x for x in p.iterdir() if x.is_file() and x.suffix.lower() == ".mkv")
        jsons = sorted(x for x in p.iterdir() if x.is_file() and x.suffix.lower() == ".json")
        if len(mkvs) != 1:
            raise RuntimeError(f"expected exactly one MKV in {p}, found {len(mkvs)}")
        if len(jsons) > 1:
            raise RuntimeError(f"expected at most one manifest in {p}, found {len(jsons)}")
        mkv, man = mkvs[0], (jsons[0] if jsons else None)
    elif p.suffix.lower() == ".json":
        m = read_manifest(p)
        cand = [Path(m["staged_mkv"]).expanduser().resolve()] if m.get("staged_mkv") else []
        cand.append(p.with_suffix(".mkv"))
        mkv = next((c for c in cand if c.exists()), None)
        if mkv is None:
            raise RuntimeError(f"no MKV found for manifest {p}")
        return Bundle(mkv, p, m)
    else:
        mkv, man = p, (p.with_suffix(".json") if p.with_suffix(".json").exists() else None)
    return Bundle(mkv, man, read_manifest(man) if man else {})


def unique_dir(p: Path) -> Path:
    if not p.exists():
        return p
    for i in range(2, 10000):
        q = p.with_name(f"{p.name} ({i})")
        if not q.exists():
            return q
    raise RuntimeError(f"no free directory name for {p}")


def unique_dest(p: Path, current: Path | None = None) -> Path:
    """`p`, or `p` with " (n)" before the suffix — never a different existing file (renaming
    a file onto itself is allowed)."""
    cur = current.resolve() if current is not None else None
    q, n = p, 2
    while q.exists() and q.resolve() != cur:
        q = p.with_name(f"{p.stem} ({n}){p.suffix}")
        n += 1
    return q


def bundle_name(disc_label: str, title: str) -> str:
    return f"{time.strftime('%Y%m%d-%H%M%S')} {safe_filename(disc_label or title or FALLBACK_TITLE)}"


def stage(finished: Path, manifest: dict, staging_root: Path, disc_label: str, title: str) -> Bundle:
    """Move a finished rip into a new staging bundle with a pending-review manifest."""
    staging_root.mkdir(parents=True, exist_ok=True)
    d = unique_dir(staging_root / bundle_name(disc_label, title))
    d.mkdir(parents=True)
    mkv = d / finished.name
    shutil.move(str(finished), mkv)
    m = {**manifest, "staged_mkv": str(mkv), "review_status": "pending", "staged_at_epoch": time.time()}
    man = mkv.with_suffix(".json")
    write_manifest(man, m)
    return Bundle(mkv, man, m)


def remove_if_empty(d: Path) -> None:
    try:
        d.rmdir()
    except OSError:
        pass


def finalize(b: Bundle, final: Path, manifest: dict, mode: str) -> Bundle:
    """Move the bundle's MKV to `final` and write its manifest beside it.  mode: "new" (fresh
    confident rip), "staged" (resolving a staged bundle) or "rename" (correcting a finished
    rip).  The old manifest / empty bundle directory is removed."""
    final.parent.mkdir(parents=True, exist_ok=True)
    src = b.mkv
    if src.resolve() != final.resolve():
        shutil.move(str(src), final)
    now = time.time()
    m = dict(manifest)
    m.pop("staged_mkv", None)
    if mode == "rename":
        m.update(review_status="corrected", corrected_at_epoch=now, original_filename=src.name)
    else:
        m["review_status"] = "resolved" if mode == "staged" else "not_needed"
    m.update(resolved_at_epoch=now, final_filename=final.name)
    man = final.with_suffix(".json")
    write_manifest(man, m)
    if b.manifest_path is not None and b.manifest_path.resolve() != man.resolve() and b.manifest_path.exists():
        b.manifest_path.unlink()
    if mode in ("staged", "rename"):
        remove_if_empty(src.parent)
    return Bundle(final, man, m)
