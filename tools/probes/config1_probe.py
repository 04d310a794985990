"""BASELINE config 1 (one 8 s WAV through the drop-in main.parse): ms per call over recurrence
options of the Model's engine, interleaved rounds (env OPTS: ';'-separated CASR_OPTS-style sets,
'-' = defaults); the text must not change."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))
sys.path.insert(0, REPO)
import main as casr_main  # noqa: E402
import model as casr_model  # noqa: E402
from data import AudioBase  # noqa: E402
from casr.config import CasrConfig  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402

m = casr_model.Model()
m.load_state_dicts(*synthetic_state_dicts(CasrConfig(), peaked=True, eos_bias=0.0))
ab = AudioBase()
wav = (0.1 * np.random.RandomState(99).standard_normal(8 * 16000 + 512)).astype(np.float32)
sets = [s for s in os.environ.get("OPTS", "-;REC_LAYOUT=2").split(";")]
defaults = {n: m.engine.get_option(n) for s in sets if s != "-" for n, _ in (kv.split("=") for kv in s.split(","))}
ref = None
for rnd in range(3):
    for s in sets:
        for n, v in defaults.items():
            m.engine.set_option(n, v)
        if s != "-":
            for kv in s.split(","):
                n, v = kv.split("=")
                m.engine.set_option(n, int(v))
        text = casr_main.parse(wav, m, ab, None, None)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            text = casr_main.parse(wav, m, ab, None, None)
        dt = (time.perf_counter() - t0) / 20
        ref = text if ref is None else ref
        assert text == ref, (s, text, ref)
        print(f"[{rnd}] {s}: {1000 * dt:.3f} ms per call", flush=True)
print("text equal across options: yes")
