"""Frozen model/decoder configuration read from the reference's ``gpd`` keys.

The reference binds these values at import time into class attributes and default
arguments (encoder.py:17-24, decoder.py:11-16, attention.py:21, model.py:606-610).
Here they are frozen once into a plain struct that is handed to the C-ABI at handle
creation (``casr_config`` in include/casr.h).
"""
from dataclasses import dataclass, asdict


@dataclass(frozen=True)
class CasrConfig:
    n_mels: int = 80            # gpd.py:13
    delta_delta: bool = True    # gpd.py:18
    downsample: bool = True     # gpd.py:19
    enc_hidden: int = 256       # gpd.py:64
    enc_layers: int = 4         # gpd.py:65
    residual: bool = True       # gpd.py:66
    dec_hidden: int = 512       # gpd.py:80
    embed_dim: int = 256        # gpd.py:82
    attn_size: int = 128        # gpd.py:89
    max_num_words: int = 5000   # gpd.py:47
    max_len: int = 40           # gpd.py:125
    pad: int = 0                # gpd.py:39
    sos: int = 1                # gpd.py:40
    eos: int = 2                # gpd.py:41
    temperature: float = 1.0    # gpd.py:83 (main.py:125 sets 1)

    @property
    def feat_dim(self):
        # encoder.py:19: n_mels * (3 if downsample) * (3 if delta_delta)
        return self.n_mels * (3 if self.downsample else 1) * (3 if self.delta_delta else 1)

    @property
    def vocab(self):
        # decoder.py:11-12: real_vcb_sz = max_num_words + 4
        return self.max_num_words + 4

    @property
    def enc_size(self):
        return 2 * self.enc_hidden

    def as_dict(self):
        d = asdict(self)
        d.update(feat_dim=self.feat_dim, vocab=self.vocab)
        return d


def config_from_gpd(gpd):
    """Build the frozen config from a reference-style ``gpd`` dict, rejecting the settings
    this MI355X path does not implement (it covers the deployed LSTM/Bahdanau config)."""
    unsupported = []
    if gpd.get('encoder_type', 'LSTM') != 'LSTM':
        unsupported.append('encoder_type')
    if not gpd.get('encoder_bidirectional', True):
        unsupported.append('encoder_bidirectional')
    if gpd.get('skip_step', 0) != 0:
        unsupported.append('skip_step')
    if gpd.get('decoder_type', 'LSTM') != 'LSTM' or gpd.get('decoder_num_layers', 1) != 1:
        unsupported.append('decoder_type/decoder_num_layers')
    if gpd.get('attn_type', 'B') != 'B' or gpd.get('heads', 1) != 1 or gpd.get('map_enc', False):
        unsupported.append('attn_type/heads/map_enc')
    if not gpd.get('input_feeding', True) or gpd.get('dec_init_cell_state_as_param', False):
        unsupported.append('input_feeding/dec_init_cell_state_as_param')
    if not gpd.get('delta_delta', True) or not gpd.get('downsample', True):
        unsupported.append('delta_delta/downsample')
    if unsupported:
        raise NotImplementedError(f"casr MI355X path does not implement gpd settings: {unsupported}")
    return CasrConfig(
        n_mels=gpd.get('n_mels', 80),
        enc_hidden=gpd.get('encoder_hidden_size', 256),
        enc_layers=gpd.get('encoder_num_layers', 4),
        residual=gpd.get('residual', True),
        dec_hidden=gpd.get('decoder_hidden_size', 512),
        embed_dim=gpd.get('embed_dim', 256),
        attn_size=gpd.get('attn_size', 128),
        max_num_words=gpd.get('max_num_words', 5000),
        max_len=gpd.get('max_len', 40),
        pad=gpd.get('pad', 0), sos=gpd.get('sos', 1), eos=gpd.get('eos', 2),
        temperature=float(gpd.get('temperature', 1.0)),
    )
