"""Drop-in for the reference's global config dict ``gpd`` (gpd.py:4-133).

Only the keys the inference path reads are kept, with the reference defaults.  As in the
reference, ``Model()`` reads them when it is constructed (the reference binds several at
import time: encoder.py:17-24, decoder.py:11-16, model.py:606-610); ``main.py`` overrides
``verbose``, ``use_cuda`` and ``temperature`` (main.py:122-125).
"""
gpd = {
    'verbose': True,
    # audio / features (data.py)
    'sample_rate': 16000,
    'window_len': .025,
    'window_step': .01,
    'n_mels': 80,
    'preemphasis': .97,
    'delta_delta': True,
    'downsample': True,
    'normalize': True,
    # dictionary
    'pad': 0,
    'sos': 1,
    'eos': 2,
    'unk': 3,
    'max_num_words': 5000,
    # encoder
    'encoder_type': 'LSTM',
    'skip_step': 0,
    'encoder_hidden_size': 256,
    'encoder_num_layers': 4,
    'residual': True,
    'encoder_bidirectional': True,
    # decoder
    'decoder_type': 'LSTM',
    'decoder_hidden_size': 512,
    'decoder_num_layers': 1,
    'embed_dim': 256,
    'temperature': 1.,
    'input_feeding': True,
    'dec_init_cell_state_as_param': False,
    # attention
    'attn_type': 'B',
    'attn_size': 128,
    'map_enc': False,
    'heads': 1,
    'linear_map': False,
    # eval / decode
    'eval_batch_size': 256,
    'beam_width': 4,
    'lm_path': '/data/zh_giga.no_cna_cmn.prune01244.klm',
    'second_pass': True,
    'max_len': 40,
    'lm_weight': 0.0,
    'length_weight': 0.0,
    # device: the MI355X path always runs on the GPU; kept for callers that set it
    'use_cuda': True,
}
