"""DVD rip/queue decision logic with recorded-style MakeMKV robot output and a fake TMDb
(no makemkvcon, no network; parity unpinned: the reference ships no fixtures)."""
import json
import shutil
from pathlib import Path

import pytest

from thinvids_amd import rips
from thinvids_amd.rips import bundle, cli, select, tools

ROBOT = """MSG:1005,0,1,"MakeMKV v1.17 started","%1 started","MakeMKV v1.17"
CINFO:1,6209,"DVD disc"
CINFO:2,0,"THE_MATRIX_16X9"
CINFO:32,0,"THE_MATRIX"
TINFO:0,2,0,"The Matrix"
TINFO:0,8,0,"32"
TINFO:0,9,0,"2:16:17"
TINFO:0,11,0,"7340032000"
TINFO:0,16,0,"01.mpls"
TINFO:0,27,0,"The_Matrix_t00.mkv"
TINFO:1,9,0,"0:02:10"
TINFO:1,11,0,"104857600"
TINFO:2,9,0,"1:05:00"
TINFO:2,11,0,"2000000000"
SINFO:0,0,1,6201,"Video"
SINFO:0,0,19,0,"720x480"
SINFO:0,1,1,6202,"Audio"
SINFO:0,1,3,0,"fra"
SINFO:0,2,1,6202,"Audio"
SINFO:0,2,3,0,"eng"
SINFO:0,3,1,6203,"Subtitles"
SINFO:0,3,3,0,"eng"
SINFO:0,4,1,6203,"Subtitles"
SINFO:0,4,3,0,"spa"
"""


def test_parse_and_choose():
    p = rips.parse_makemkv_robot_output(ROBOT)
    assert [t["index"] for t in p["titles"]] == [0, 2, 1]
    t = rips.choose_main_title(p, min_seconds=2400)
    assert t["index"] == 0 and t["duration_seconds"] == 2 * 3600 + 16 * 60 + 17 and t["chapters_count"] == 32
    assert len(t["streams"]) == 5 and t["streams"][0]["video_size"] == "720x480"
    assert p["disc_info"]["2"] == "THE_MATRIX_16X9"
    assert rips.choose_main_title({"titles": [{"index": 3, "duration_seconds": 60}]})["index"] == 3


def test_hints_cleanup_and_generic():
    assert rips.split_title_year_hint("THE_MATRIX_16X9 (1999)") == ("THE MATRIX", "1999")
    assert rips.is_generic_hint("DVD_VIDEO") and rips.is_low_information_hint("AB12")
    p = rips.parse_makemkv_robot_output(ROBOT)
    hints = rips.build_auto_title_hints(p, rips.choose_main_title(p), disc_label="THE_MATRIX_WS")
    assert hints[0]["source"] == "disc-label" and hints[0]["query"] == "THE MATRIX"
    assert len({rips.normalize_title(h["query"]) for h in hints}) == len(hints)  # deduplicated


def test_tmdb_scoring_and_review_threshold():
    db = {"/search/movie": {"results": [{"id": 1, "title": "The Matrix", "release_date": "1999-03-30"},
                                        {"id": 2, "title": "The Matrix Reloaded", "release_date": "2003-05-15"}]},
          "/movie/1": {"runtime": 136}, "/movie/2": {"runtime": 138}}
    tm = rips.Tmdb("k", fetch=lambda path, params: db.get(path))
    p = rips.parse_makemkv_robot_output(ROBOT)
    t = rips.choose_main_title(p)
    meta = rips.auto_detect_movie_metadata(p, t, disc_label="THE_MATRIX", tmdb=tm)
    assert meta["title"] == "The Matrix" and meta["year"] == "1999" and not meta["needs_manual_review"]
    low = rips.auto_detect_movie_metadata(p, t, disc_label="THE_MATRIX", tmdb=tm, min_score=500)
    assert low["needs_manual_review"] and "score" in low["review_reason"]
    off = rips.auto_detect_movie_metadata(p, t, disc_label="THE_MATRIX", tmdb=None)
    assert off["needs_manual_review"] and off["title"] == "The Matrix"
    assert rips.runtime_adjustment(8177, 136) > rips.runtime_adjustment(8177, 90)


def test_paths_streams_and_staging(tmp_path):
    f = rips.build_final_path(tmp_path, "The Matrix: Reloaded?", "2003", 480)
    assert f == tmp_path / "movies" / "The Matrix Reloaded (2003)" / "The Matrix Reloaded (2003) 480p h264.mkv"
    f.parent.mkdir(parents=True)
    f.write_bytes(b"x")
    assert rips.build_final_path(tmp_path, "The Matrix: Reloaded?", "2003", 480).name.endswith("[2].mkv")
    p = rips.parse_makemkv_robot_output(ROBOT)
    plan = rips.remux_plan(rips.choose_main_title(p)["streams"])
    assert plan == {"video": [0], "audio": [2], "subtitles": [3]}
    mkv = tmp_path / "title_t00.mkv"
    mkv.write_bytes(b"rip")
    staged = rips.stage_for_manual_review(mkv, tmp_path / "staging", {"title": "x", "needs_manual_review": True})
    assert staged.exists() and Path(str(staged.with_suffix(".json"))).exists() and not mkv.exists()
    assert staged.parent.parent == tmp_path / "staging"  # one bundle directory per staged rip
    sent = {}

    class R:
        def json(self):
            return {"status": "success"}

    def post(url, json, timeout):
        sent.update(url=url, json=json)
        return R()

    assert rips.submit_add_job("http://m:5005/", "movies/x.mkv", post=post)["status"] == "success"
    assert sent["url"] == "http://m:5005/add_job" and sent["json"]["mark_watcher_processed"] is True


# ------------------------------------------------------------------ full CLI flow

PROGRESS = ['PRGT:5018,0,"Saving to MKV file"', 'PRGC:5018,0,"Saving to MKV file"', 'PRGC:5017,0,"Analyzing seamless segments"']
PROGRESS += [f"PRGV:{c},{c // 2},65536" for c in range(0, 65537, 1024)]
FFPROBE = {"streams": [{"index": 0, "codec_type": "video", "codec_name": "mpeg2video", "width": 720, "height": 480},
                       {"index": 1, "codec_type": "audio", "codec_name": "ac3", "channels": 6, "tags": {"language": "fre"}},
                       {"index": 2, "codec_type": "audio", "codec_name": "ac3", "channels": 6, "tags": {"language": "eng"}},
                       {"index": 3, "codec_type": "subtitle", "codec_name": "dvd_subtitle", "tags": {"language": "eng"}},
                       {"index": 4, "codec_type": "subtitle", "codec_name": "dvd_subtitle", "tags": {"language": "spa"}}]}


class FakeTools(tools.Runner):
    """Recorded makemkvcon / ffprobe / ffmpeg / blkid behaviour."""

    def __init__(self, have=("makemkvcon", "ffmpeg", "ffprobe", "blkid"), label="THE_MATRIX"):
        self.have, self.label, self.calls = set(have), label, []

    def which(self, name):
        return name in self.have

    def run(self, cmd):
        self.calls.append(cmd)
        if cmd[0] == "makemkvcon":
            return tools.Result(0, 'DRV:0,2,999,1,"BD-RE","THE_MATRIX","/dev/sr7"\nDRV:1,256,999,0,"","",""\n')
        if cmd[0] == "blkid":
            return tools.Result(0, self.label + "\n")
        if cmd[0] == "ffprobe":
            return tools.Result(0, json.dumps(FFPROBE))
        if cmd[0] == "ffmpeg":
            shutil.copyfile(cmd[cmd.index("-i") + 1], cmd[-1])
            return tools.Result(0)
        return tools.Result(127)

    def lines(self, cmd):
        self.calls.append(cmd)
        if "mkv" in cmd:
            out = Path(cmd[-1])
            (out / "title_t00.mkv").write_bytes(b"\x1aE\xdf\xa3 fake matroska")
            return iter(PROGRESS), lambda: 0
        return iter(ROBOT.splitlines() + PROGRESS[:3]), lambda: 0


TMDB = {"/search/movie": {"results": [{"id": 1, "title": "The Matrix", "release_date": "1999-03-30"}]},
        "/movie/1": {"runtime": 136}}


def _args(tmp_path, *extra):
    a = cli.build_parser({}).parse_args(["--watch-root", str(tmp_path / "watch"), "--scratch-root", str(tmp_path / "scr"),
                                         "--staging-root", str(tmp_path / "stg"), "--tmdb-api-key", "k", *extra])
    return a


def _tmdb(key):
    return rips.Tmdb(key, fetch=lambda path, params: TMDB.get(path))


def test_cli_confident_rip_is_finalised_and_queued(tmp_path):
    ft, posted, msgs = FakeTools(), {}, []

    class R:
        def json(self):
            return {"status": "success", "job_id": "j1"}

    def post(url, json, timeout):
        posted.update(url=url, json=json)
        return R()

    out = cli.run(_args(tmp_path, "--queue-mode", "api", "--device", "/dev/sr7"), runner=ft, tmdb_factory=_tmdb,
                  sink=msgs.append, post=post)
    final = Path(out["final_path"])
    assert final == tmp_path / "watch/movies/The Matrix (1999)/The Matrix (1999) 480p h264.mkv" and final.exists()
    man = json.loads(final.with_suffix(".json").read_text())
    assert man["review_status"] == "not_needed" and man["disc_label"] == "THE_MATRIX" and man["english_subtitles_kept"]
    assert posted["json"] == {"filename": "movies/The Matrix (1999)/The Matrix (1999) 480p h264.mkv",
                              "mark_watcher_processed": True} and out["api_result"]["job_id"] == "j1"
    assert not list((tmp_path / "scr").iterdir())  # temp rip dir removed
    # source resolved from the drive scan; default remux maps: all video, English AC-3, English subtitle
    assert ["makemkvcon", "--robot", "--progress=-same", "mkv", "disc:0", "0"] == [c for c in ft.calls if "mkv" in c][0][:6]
    ff = [c for c in ft.calls if c[0] == "ffmpeg"][0]
    assert ff[ff.index("-i") + 2:ff.index("-map_metadata")] == ["-map", "0:v", "-map", "0:2", "-map", "0:3"]
    # progress: ~20 overall steps, not one line per PRGV record
    prog = [m for m in msgs if "rip title" in m and "%" in m]
    assert 10 <= len(prog) <= 25 and prog[-1].endswith("(50% overall, 100% current)")


def test_cli_low_confidence_is_staged_then_resumed_and_renamed(tmp_path):
    ft = FakeTools()
    out = cli.run(_args(tmp_path, "--auto-title-min-score", "1000"), runner=ft, tmdb_factory=_tmdb, sink=lambda m: None)
    assert out["manual_review_required"] and out["final_path"] == ""
    staged = Path(out["staged_path"])
    man = json.loads(staged.with_suffix(".json").read_text())
    assert man["review_status"] == "pending" and man["staged_mkv"] == str(staged) and "score" in man["review_reason"]
    assert staged.parent.parent == tmp_path / "stg"
    # resume from the bundle directory with a corrected title: no drive access
    ft2 = FakeTools(have=("ffprobe",))
    out2 = cli.run(_args(tmp_path, "Matrix", "--staged-path", str(staged.parent)), runner=ft2, tmdb_factory=_tmdb,
                   sink=lambda m: None)
    final = Path(out2["final_path"])
    assert final.exists() and final.parent.name == "The Matrix (1999)" and not staged.parent.exists()
    m2 = json.loads(final.with_suffix(".json").read_text())
    assert m2["review_status"] == "resolved" and m2["disc_label"] == "THE_MATRIX" and "staged_mkv" not in m2
    assert not any(c[0] == "makemkvcon" for c in ft2.calls)
    # rename the finished rip in place (given its manifest); no re-queue
    out3 = cli.run(_args(tmp_path, "Bound (1996)", "--rename-path", str(final.with_suffix(".json"))),
                   runner=FakeTools(have=("ffprobe",)), tmdb_factory=lambda k: None, sink=lambda m: None)
    f3 = Path(out3["rename_path"])
    assert f3.name == "Bound (1996) 480p h264.mkv" and f3.exists() and not final.exists()
    m3 = json.loads(f3.with_suffix(".json").read_text())
    assert m3["review_status"] == "corrected" and m3["original_filename"] == final.name
    assert not final.with_suffix(".json").exists() and out3["api_result"] is None


def test_cli_validation_dry_run_and_diagnostic(tmp_path):
    with pytest.raises(SystemExit, match="makemkvcon"):
        cli.run(_args(tmp_path), runner=FakeTools(have=()))
    with pytest.raises(SystemExit, match="cannot be used together"):
        cli.run(_args(tmp_path, "x", "--staged-path", "a", "--rename-path", "b"), runner=FakeTools())
    with pytest.raises(SystemExit, match="explicit title"):
        cli.run(_args(tmp_path, "--staged-path", "a"), runner=FakeTools())
    with pytest.raises(SystemExit, match="title-index"):
        cli.run(_args(tmp_path, "x", "--staged-path", "a", "--title-index", "1"), runner=FakeTools())
    plan = cli.run(_args(tmp_path, "--dry-run", "--title-index", "2"), runner=FakeTools(), tmdb_factory=_tmdb,
                   sink=lambda m: None)
    assert plan["selected_title"]["index"] == 2 and plan["output_path"].endswith("<resolution> h264.mkv")
    assert not (tmp_path / "watch").exists()

    class Empty(FakeTools):
        def lines(self, cmd):
            return iter(['MSG:5010,0,0,"Failed to open disc"']), lambda: 0

    with pytest.raises(SystemExit, match="no titles"):
        cli.run(_args(tmp_path), runner=Empty(), sink=lambda m: None)
    assert list((tmp_path / "scr").glob("makemkv-info-*.log"))
    with pytest.raises(SystemExit):
        cli.build_parser({}).parse_args(["--output-subdir", "../x"])


def test_interactive_selection(tmp_path):
    p = rips.parse_makemkv_robot_output(ROBOT)
    t = rips.choose_main_title(p)
    answers = iter(["9", "2"])
    picked = select.choose_title(p, t, ask=lambda q: next(answers), out=lambda m: None, tty=lambda: True)
    assert picked["index"] == p["titles"][1]["index"]
    with pytest.raises(RuntimeError, match="terminal"):
        select.choose_title(p, t, tty=lambda: False)
    # video: Enter (default), audio: "1" (French), subtitles: "none"
    answers = iter(["", "x", "1", "none"])
    specs = select.choose_streams(t["streams"], ask=lambda q: next(answers), out=lambda m: None, tty=lambda: True)
    assert specs == [{"codec_type": "video", "ordinal": 0}, {"codec_type": "audio", "ordinal": 0}]
    assert select.parse_menu("1,2,2", [1, 2, 3], multiple=True) == [1, 2] and select.parse_menu("4", [1]) is None
    # picks map onto the ripped file's ffprobe numbering, and drive the ffmpeg maps
    ft = FakeTools()
    chosen = tools.resolve_selection(ft, specs, tmp_path / "x.mkv")
    assert [s["index"] for s in chosen] == [0, 1]
    src = tmp_path / "in.mkv"
    src.write_bytes(b"x")
    assert tools.remux(ft, src, tmp_path / "out.mkv", "T", chosen) is False
    assert [c for c in ft.calls if c[0] == "ffmpeg"][0].count("-map") == 2
    assert tools.remux(FakeTools(have=()), src, tmp_path / "o2.mkv", "T") is None


def test_drive_scan_label_and_config(tmp_path, monkeypatch):
    ft = FakeTools()
    assert tools.resolve_source(ft, "auto", "/dev/sr7") == "disc:0" and tools.resolve_source(ft, "disc:3", "x") == "disc:3"
    assert tools.resolve_source(ft, "auto", "/dev/sr9") == "disc:0"
    assert tools.parse_drive_scan('DRV:1,2,999,1,"a","b","/dev/sr1"')[0]["device_path"] == "/dev/sr1"
    assert tools.probe_disc_label(ft, "/dev/sr7") == "THE_MATRIX"
    env = tmp_path / "defaults"
    env.write_text('# c\nexport THINVIDS_DVD_QUEUE_MODE="api"\nTHINVIDS_DVD_MIN_SECONDS=600\nBAD LINE\n')
    cfg = rips.load_env_file(env)
    assert cfg == {"THINVIDS_DVD_QUEUE_MODE": "api", "THINVIDS_DVD_MIN_SECONDS": "600"}
    monkeypatch.setenv("THINVIDS_DVD_MIN_SECONDS", "900")
    a = cli.build_parser(cfg).parse_args([])
    assert a.queue_mode == "api" and a.min_seconds == 900  # environment beats the file
    assert rips.configured({"X": "abc"}, "X", fallback=5, cast=int) == 5


def test_bundle_locate_forms(tmp_path):
    d = tmp_path / "b"
    d.mkdir()
    (d / "m.mkv").write_bytes(b"1")
    assert bundle.locate(d).mkv == d / "m.mkv" and bundle.locate(d).manifest_path is None
    bundle.write_manifest(d / "m.json", {"k": 1})
    assert bundle.locate(d / "m.mkv").manifest == {"k": 1} and bundle.locate(d / "m.json").mkv == d / "m.mkv"
    (d / "n.mkv").write_bytes(b"2")
    with pytest.raises(RuntimeError, match="exactly one MKV"):
        bundle.locate(d)
    with pytest.raises(RuntimeError, match="does not exist"):
        bundle.locate(tmp_path / "nope")
    f = tmp_path / "a.mkv"
    f.write_bytes(b"x")
    assert bundle.unique_dest(f) == tmp_path / "a (2).mkv" and bundle.unique_dest(f, current=f) == f
