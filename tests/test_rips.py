"""DVD rip/queue decision logic with recorded-style MakeMKV robot output and a fake TMDb
(no makemkvcon, no network; parity unpinned: the reference ships no fixtures)."""
from pathlib import Path

from thinvids_amd import rips

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
    sent = {}

    class R:
        def json(self):
            return {"status": "success"}

    def post(url, json, timeout):
        sent.update(url=url, json=json)
        return R()

    assert rips.submit_add_job("http://m:5005/", "movies/x.mkv", post=post)["status"] == "success"
    assert sent["url"] == "http://m:5005/add_job" and sent["json"]["mark_watcher_processed"] is True
