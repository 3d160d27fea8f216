"""/system inventory (pkg/xsysinfo): CPU flags from procfs, AMD GPUs + VRAM from amdgpu sysfs."""
from localai_amd.utils import sysinfo


def test_gpu_inventory_from_sysfs(tmp_path):
    for card, vendor in (("card0", "0x1002"), ("card1", "0x8086")):
        d = tmp_path / card / "device"
        d.mkdir(parents=True)
        (d / "vendor").write_text(vendor + "\n")
        (d / "device").write_text("0x75a3\n")
        (d / "mem_info_vram_total").write_text(str(288 << 30) + "\n")
        (d / "mem_info_vram_used").write_text("1024\n")
    (tmp_path / "card0-DP-1").mkdir()
    g = sysinfo.gpus(str(tmp_path))
    assert len(g) == 1 and g[0]["card"] == "card0" and g[0]["vram_total"] == 288 << 30
    assert g[0]["vram_used"] == 1024 and g[0]["device_id"] == "0x75a3"


def test_cpu_capabilities(tmp_path):
    f = tmp_path / "cpuinfo"
    f.write_text("processor : 0\nmodel name : AMD EPYC 9575F\nflags : fpu sse avx avx2 fma avx512f\n\n"
                 "processor : 1\nmodel name : AMD EPYC 9575F\nflags : fpu\n")
    c = sysinfo.cpu_info(str(f))
    assert c["model"] == "AMD EPYC 9575F" and c["capabilities"] == ["avx", "avx2", "avx512f", "fma"]
    assert "cpu" in sysinfo.system_info()

