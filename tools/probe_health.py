"""What GPU health sources are readable on this box (ECC / RAS / xGMI)?

Prints sysfs RAS counter readability and the amdsmi ECC / xGMI readings of
GPU 0, so the runtime's health monitor (Backend::device_health) can pick a
source that works (reference: uvm_gpu.c:1328-1354, 2087-2104).
"""
from __future__ import annotations

import glob
import os


def sysfs() -> None:
    for d in sorted(glob.glob("/sys/bus/pci/drivers/amdgpu/*/ras"))[:2]:
        files = sorted(os.listdir(d))
        print("sysfs", d, files)
        for f in files:
            p = os.path.join(d, f)
            try:
                with open(p) as fh:
                    print("  ", f, repr(fh.read()[:120]))
            except OSError as e:
                print("  ", f, "unreadable:", e)


def smi() -> None:
    import amdsmi as A

    A.amdsmi_init(A.AmdSmiInitFlags.INIT_AMD_GPUS)
    hs = A.amdsmi_get_processor_handles()
    print("amdsmi gpus", len(hs))
    h = hs[0]
    for name, fn in [
        ("bdf", lambda: A.amdsmi_get_gpu_device_bdf(h)),
        ("ecc_enabled", lambda: A.amdsmi_get_gpu_ecc_enabled(h)),
        ("total_ecc", lambda: A.amdsmi_get_gpu_total_ecc_count(h)),
        ("ecc_umc", lambda: A.amdsmi_get_gpu_ecc_count(h, A.AmdSmiGpuBlock.UMC)),
        ("ecc_xgmi", lambda: A.amdsmi_get_gpu_ecc_count(h, A.AmdSmiGpuBlock.XGMI_WAFL)),
        ("ecc_status_umc", lambda: A.amdsmi_get_gpu_ecc_status(h, A.AmdSmiGpuBlock.UMC)),
        ("xgmi_error_status", lambda: A.amdsmi_gpu_xgmi_error_status(h)),
        ("xgmi_link_status", lambda: A.amdsmi_get_gpu_xgmi_link_status(h)),
        ("xgmi_info", lambda: A.amdsmi_get_xgmi_info(h)),
    ]:
        try:
            print("  ", name, fn())
        except Exception as e:  # noqa: BLE001 - probing what the box supports
            print("  ", name, "ERROR", type(e).__name__, e)
    A.amdsmi_shut_down()


if __name__ == "__main__":
    sysfs()
    try:
        smi()
    except Exception as e:  # noqa: BLE001
        print("amdsmi unavailable:", e)
