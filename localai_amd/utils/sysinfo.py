"""Host and GPU inventory for `/system` and the backend monitor (pkg/xsysinfo/cpu.go:10-45,
gpu.go:8-15: CPU capability flags and the GPU list).

Read from procfs/sysfs only: asking HIP would create a device context in the gateway process
(hundreds of MiB of HBM per GPU) just to answer a status request."""
from __future__ import annotations

import glob
import os
from typing import Dict, List

_CPU_FLAGS = ("avx", "avx2", "avx512f", "avx512_bf16", "amx_bf16", "fma", "f16c")


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return ""


def cpu_info(cpuinfo: str = "/proc/cpuinfo") -> Dict:
    model, flags = "", set()
    for line in _read(cpuinfo).splitlines():
        k, _, v = line.partition(":")
        k = k.strip()
        if k == "model name" and not model:
            model = v.strip()
        elif k == "flags" and not flags:
            flags = set(v.split())
    return {"model": model, "cores": os.cpu_count() or 0,
            "capabilities": [f for f in _CPU_FLAGS if f in flags]}


def gpus(drm_root: str = "/sys/class/drm") -> List[Dict]:
    """AMD GPUs (PCI vendor 0x1002) with VRAM totals from the amdgpu sysfs nodes."""
    out = []
    for card in sorted(glob.glob(os.path.join(drm_root, "card[0-9]*"))):
        if "-" in os.path.basename(card):  # connectors (card0-DP-1)
            continue
        dev = os.path.join(card, "device")
        if _read(os.path.join(dev, "vendor")).lower() != "0x1002":
            continue
        total = _read(os.path.join(dev, "mem_info_vram_total"))
        used = _read(os.path.join(dev, "mem_info_vram_used"))
        out.append({"card": os.path.basename(card), "vendor": "AMD",
                    "device_id": _read(os.path.join(dev, "device")),
                    "product": _read(os.path.join(dev, "product_name")) or None,
                    "vram_total": int(total) if total.isdigit() else None,
                    "vram_used": int(used) if used.isdigit() else None})
    return out


def system_info() -> Dict:
    return {"cpu": cpu_info(), "gpus": gpus()}
