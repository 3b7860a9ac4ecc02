"""MI355X GPU sampler for the node agent (replaces the reference's
``intel_gpu_top -J`` video-engine busy %, agent/agent.py:42-117).

Uses the ``amdsmi`` Python API (graphics activity, VRAM/HBM used/total, power, edge
temperature, market name, accumulated xGMI read / write bytes over all links) and falls
back to ``rocm-smi --json`` when the library cannot be initialised.  The xGMI totals are
monotonically increasing byte counters; the agent turns them into per-second rates the
same way it does for the NIC (reference payload ``rx_bps`` / ``tx_bps``,
agent/agent.py:410-429).  Returns ``None`` when no AMD GPU is visible (the agent then publishes
``gpu = -1`` exactly like the reference did without an iGPU).
"""
from __future__ import annotations

import json
import logging
import shutil
import subprocess

log = logging.getLogger("thinvids.agent.gpu")


def _num(v, d=0.0):
    try:
        if isinstance(v, dict):
            v = v.get("value", d)
        return float(v)
    except (TypeError, ValueError):
        return d


class GpuSampler:
    def __init__(self):
        self._smi = None
        self._handles = []
        try:
            import amdsmi

            amdsmi.amdsmi_init()
            self._handles = list(amdsmi.amdsmi_get_processor_handles() or [])
            self._smi = amdsmi if self._handles else None
        except Exception as e:  # no driver / no device (CPU-only host)
            log.debug("amdsmi unavailable: %s", e)
            self._smi = None

    def _amdsmi_sample(self) -> list[dict]:
        smi = self._smi
        out = []
        for i, h in enumerate(self._handles):
            g = {"index": i}
            try:
                act = smi.amdsmi_get_gpu_activity(h)
                g["util"] = _num(act.get("gfx_activity"))
                g["mem_util"] = _num(act.get("umc_activity"))
            except Exception:
                g["util"] = -1.0
            try:
                g["hbm_total"] = int(smi.amdsmi_get_gpu_memory_total(h, smi.AmdSmiMemoryType.VRAM))
                g["hbm_used"] = int(smi.amdsmi_get_gpu_memory_usage(h, smi.AmdSmiMemoryType.VRAM))
            except Exception:
                pass
            try:
                g["name"] = smi.amdsmi_get_gpu_asic_info(h).get("market_name", "")
            except Exception:
                g["name"] = ""
            try:
                p = smi.amdsmi_get_power_info(h)
                g["power_w"] = _num(p.get("current_socket_power", p.get("average_socket_power")))
            except Exception:
                pass
            rd, wr = xgmi_bytes(smi, h)
            if rd is not None:
                g["xgmi_read_bytes"], g["xgmi_write_bytes"] = rd, wr
            try:
                g["temp_c"] = _num(smi.amdsmi_get_temp_metric(h, smi.AmdSmiTemperatureType.HOTSPOT,
                                                               smi.AmdSmiTemperatureMetric.CURRENT))
            except Exception:
                pass
            out.append(g)
        return out

    @staticmethod
    def _rocm_smi_sample() -> list[dict]:
        exe = shutil.which("rocm-smi")
        if not exe:
            return []
        try:
            r = subprocess.run([exe, "--showuse", "--showmeminfo", "vram", "--showproductname", "--json"],
                               capture_output=True, text=True, timeout=5)
            data = json.loads(r.stdout or "{}")
        except (OSError, subprocess.TimeoutExpired, ValueError):
            return []
        return parse_rocm_smi(data)

    def sample(self) -> dict | None:
        gpus = self._amdsmi_sample() if self._smi else self._rocm_smi_sample()
        if not gpus:
            return None
        utils = [g["util"] for g in gpus if g.get("util", -1) >= 0]
        out = {"gpu_count": len(gpus), "util": sum(utils) / len(utils) if utils else -1.0,
               "hbm_used": sum(g.get("hbm_used", 0) for g in gpus),
               "hbm_total": sum(g.get("hbm_total", 0) for g in gpus),
               "gpu_name": gpus[0].get("name", ""), "gpus": gpus}
        if any("xgmi_read_bytes" in g for g in gpus):
            out["xgmi_read_bytes"] = sum(g.get("xgmi_read_bytes", 0) for g in gpus)
            out["xgmi_write_bytes"] = sum(g.get("xgmi_write_bytes", 0) for g in gpus)
        return out


def _kb_sum(vals) -> int | None:
    """Sum of the numeric entries of an amdsmi per-link counter list (unsupported links are
    reported as "N/A" / max-uint sentinels and skipped); None when no entry is numeric."""
    tot, seen = 0, False
    for v in vals if isinstance(vals, (list, tuple)) else [vals]:
        if isinstance(v, bool) or not isinstance(v, (int, float)) or v < 0 or v >= 2 ** 63:
            continue
        tot += int(v)
        seen = True
    return tot if seen else None


def xgmi_bytes(smi, handle) -> tuple[int | None, int | None]:
    """(read, write) bytes accumulated over every xGMI link of one GPU since driver load.
    GPU metrics table first (``xgmi_read_data_acc`` / ``xgmi_write_data_acc``, KB per link),
    then the link-metrics API (``read`` / ``write``, KB per link); (None, None) if neither
    reports a number (single-GPU or PCIe-only boxes)."""
    try:
        m = smi.amdsmi_get_gpu_metrics_info(handle)
        rd, wr = _kb_sum(m.get("xgmi_read_data_acc")), _kb_sum(m.get("xgmi_write_data_acc"))
        if rd is not None and wr is not None:
            return rd * 1024, wr * 1024
    except Exception:
        pass
    try:
        lm = smi.amdsmi_get_link_metrics(handle)
        links = lm.get("links", [])[: int(lm.get("num_links", 0) or 0)]
        rd, wr = _kb_sum([x.get("read") for x in links]), _kb_sum([x.get("write") for x in links])
        if rd is not None and wr is not None:
            return rd * 1024, wr * 1024
    except Exception:
        pass
    return None, None


def parse_rocm_smi(data: dict) -> list[dict]:
    """Parse ``rocm-smi --json`` output ({"card0": {...}, ...})."""
    out = []
    for key in sorted((k for k in data if k.startswith("card")), key=lambda k: int(k[4:] or 0)):
        d = data[key]
        g = {"index": int(key[4:] or 0), "util": _num(d.get("GPU use (%)"), -1.0),
             "name": d.get("Card Series") or d.get("Card series") or d.get("Card SKU") or ""}
        if "VRAM Total Memory (B)" in d:
            g["hbm_total"] = int(_num(d["VRAM Total Memory (B)"]))
            g["hbm_used"] = int(_num(d.get("VRAM Total Used Memory (B)")))
        out.append(g)
    return out
