"""Capture variants for the RX front-end parity tests (test infrastructure): the reference's
own recorded/synthetic captures (test_rx, test_real_rx) re-embedded with different idle
prefixes, gains, DC offsets and noise, plus captures holding no packet."""
import numpy as np


def kat_streams(fe):
    """The two KAT programs' receiver inputs: test_rx = append_idle (1000 zeros) >>>
    downSample; test_real_rx = append_idle with x10 gain (test_real_rx.blk:37-65)."""
    rx = np.concatenate([np.zeros((1000, 2), np.int16), fe["rx_in"]])
    real = np.concatenate([np.zeros((1000, 2), np.int64), fe["real_in"].astype(np.int64) * 10]).astype(np.int16)
    return rx, real


def variants(fe, n, seed):
    """n captures (receiver input, downsample off) built from the two KAT captures."""
    rng = np.random.default_rng(seed)
    rx, real = kat_streams(fe)
    rx_ds = rx[1::2][: (rx.shape[0] // 8) * 4]          # downSample: odd samples of whole groups of 8
    base = [rx_ds[500:], real[1000:]]
    caps = []
    for i in range(n):
        kind = i % 5
        if kind == 4:                                    # no packet: idle noise only
            caps.append(np.clip(rng.normal(0, rng.uniform(0, 6), (int(rng.integers(300, 1500)), 2)),
                                -32768, 32767).astype(np.int16))
            continue
        src = base[kind % 2].astype(np.float64)
        gain = rng.uniform(0.5, 2.0) if kind >= 2 else 1.0
        dc = rng.integers(-40, 41, 2) if kind == 3 else np.zeros(2)
        idle = int(rng.integers(330, 900))
        if kind % 2 == 0 and i % 3 == 0:
            idle = 500 + 16 * int(rng.integers(-8, 20))    # the KAT's alignment on the 16-sample grid
        tail = int(rng.integers(0, 400))
        sig = np.concatenate([np.zeros((idle, 2)), src * gain, np.zeros((tail, 2))]) + dc
        if kind >= 1:
            sig = sig + rng.normal(0, rng.uniform(0.5, 3.0), sig.shape)
        caps.append(np.clip(np.rint(sig), -32768, 32767).astype(np.int16))
    return caps
