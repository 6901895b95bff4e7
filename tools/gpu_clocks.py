"""GPU clock readings for bench.py (make builder and driver numbers comparable).

amdsmi (the ROCm SMI library's Python binding) gives the current GFX (sclk) and memory (mclk)
clocks of the device a rank runs on.  Every call is best effort: without amdsmi or without access
to the device the readings are None and the bench line says so.
"""
import statistics
import threading
import time


class Clocks:
    def __init__(self, torch, dev_index: int):
        self.h = None
        self.why = None
        try:
            import amdsmi

            self.smi = amdsmi
            amdsmi.amdsmi_init()
            handles = amdsmi.amdsmi_get_processor_handles()
            if len(handles) == 1:
                self.h = handles[0]
            else:  # match the torch device by PCI bus
                props = torch.cuda.get_device_properties(dev_index)
                bus = getattr(props, "pci_bus_id", None)
                for h in handles:
                    bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # "dddd:bb:dd.f"
                    if bus is not None and int(bdf.split(":")[1], 16) == int(bus):
                        self.h = h
                        break
            if self.h is None:
                self.why = f"no amdsmi handle matches device {dev_index} ({len(handles)} handles)"
        except Exception as e:  # noqa: BLE001 - a missing library is a reported fact, not an error
            self.why = f"amdsmi unavailable: {type(e).__name__}: {e}"

    def read(self):
        """{'sclk_mhz', 'sclk_max_mhz', 'mclk_mhz'} now, or None."""
        if self.h is None:
            return None
        try:
            g = self.smi.amdsmi_get_clock_info(self.h, self.smi.AmdSmiClkType.GFX)
            m = self.smi.amdsmi_get_clock_info(self.h, self.smi.AmdSmiClkType.MEM)
            return {"sclk_mhz": g.get("clk"), "sclk_max_mhz": g.get("max_clk"), "mclk_mhz": m.get("clk")}
        except Exception as e:  # noqa: BLE001
            self.why = f"amdsmi_get_clock_info failed: {type(e).__name__}: {e}"
            return None

    def sample_during(self, fn, period_s: float = 0.001):
        """Run fn() while a thread reads sclk every period_s; returns (fn's result, summary)."""
        if self.h is None:
            return fn(), None
        samples, stop = [], threading.Event()

        def loop():
            while not stop.is_set():
                r = self.read()
                if r and r["sclk_mhz"] is not None:
                    samples.append(r["sclk_mhz"])
                time.sleep(period_s)

        th = threading.Thread(target=loop, daemon=True)
        th.start()
        try:
            res = fn()
        finally:
            stop.set()
            th.join()
        if not samples:
            return res, None
        return res, {"sclk_mhz_median": statistics.median(samples), "sclk_mhz_min": min(samples),
                     "sclk_mhz_max": max(samples), "samples": len(samples)}
