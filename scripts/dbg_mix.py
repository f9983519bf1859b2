import numpy as np, sys
sys.path.insert(0, '.')
import ziria_amd as Z
g = np.load('tests/golden/ref_chain.npz')
sym, off, nsym = g["mix_sym"], g["mix_off"], g["mix_nsym"]
csr = np.concatenate([off, [off[-1] + nsym[-1]]]).astype(np.int32)
pay, info, nok = Z.wifi_rx_batch(sym, csr)
meta = g["mix_meta"]; crc = g["mix_crc"]
for i in range(len(crc)):
    print(i, tuple(meta[i]), "exp", crc[i], "got", info["crc_ok"][i], "nsym", nsym[i])
