"""CPU tests of the host-side drop-in surface: constructor signatures, parameter creation
order (a seeded construction gives the reference's weights), state_dict keys (reference
checkpoints load 1:1), vocabulary handling (H1) and the fused-MLP envelope logic."""
import inspect
import os

import torch
import torch.nn as nn

import helpers as H
import rankops
from rankops import common

V = H.SMALL_VOCAB


def _emb(n, d):
    return nn.Embedding(n + 1, d)


def _ref_dcn():
    """Reference construction order, dcn.py:130-152."""
    mods = [("embeddings.userid", _emb(V["userid"], 16)), ("embeddings.device", _emb(V["device"], 2)),
            ("embeddings.authorid", _emb(V["authorid"], 4)), ("embeddings.bgm_song_id", _emb(V["bgm_song_id"], 4)),
            ("embeddings.bgm_singer_id", _emb(V["bgm_singer_id"], 4)),
            ("embeddings.manual_tag_list", _emb(V["manual_tag_list"], 4))]
    mods += [("dnn.0", nn.Linear(50, 512)), ("dnn.2", nn.Linear(512, 256)), ("dnn.4", nn.Linear(256, 128)),
             ("output_layer", nn.Linear(178, 1))]
    return mods


def _ref_deepfm():
    """deepfm.py:90-112 (embedding_dim 8, hidden 512-256-128, BN, dropout)."""
    f = ["userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id"]
    mods = [(f"first_order_embeddings.{c}", _emb(V[c], 1)) for c in f]
    mods += [(f"second_order_embeddings.{c}", _emb(V[c], 8)) for c in f]
    mods += [("deep_layers.0", nn.Linear(48, 512)), ("deep_layers.1", nn.BatchNorm1d(512)),
             ("deep_layers.4", nn.Linear(512, 256)), ("deep_layers.5", nn.BatchNorm1d(256)),
             ("deep_layers.8", nn.Linear(256, 128)), ("deep_layers.9", nn.BatchNorm1d(128)),
             ("deep_output_layer", nn.Linear(128, 1)), ("final_layer", nn.Linear(3, 1))]
    return mods


def _ref_din():
    """din.py:251-285 (dice, BN, dropout)."""
    mods = [("embeddings.userid", _emb(V["userid"], 16)), ("embeddings.device", _emb(V["device"], 2)),
            ("embeddings.authorid", _emb(V["authorid"], 4)), ("embeddings.bgm_song_id", _emb(V["bgm_song_id"], 4)),
            ("embeddings.bgm_singer_id", _emb(V["bgm_singer_id"], 4)),
            ("embeddings.manual_tag_list", _emb(V["manual_tag_list"], 4)),
            ("embeddings.feedid", _emb(V["feedid"], 16)), ("embeddings.his_read_comment_7d_seq", _emb(V["feedid"], 16))]
    mods += [("fcn.0", nn.Linear(82, 512)), ("fcn.4", nn.Linear(512, 256)), ("fcn.8", nn.Linear(256, 128)),
             ("output_layer", nn.Linear(128, 1))]
    return mods


def _ref_bst():
    """bst.py:181-214 (d_model 16, max_len 51, BN)."""
    mods = [("embeddings.userid", _emb(V["userid"], 16)), ("embeddings.device", _emb(V["device"], 2)),
            ("embeddings.authorid", _emb(V["authorid"], 4)), ("embeddings.bgm_song_id", _emb(V["bgm_song_id"], 4)),
            ("embeddings.bgm_singer_id", _emb(V["bgm_singer_id"], 4)),
            ("embeddings.manual_tag_list", _emb(V["manual_tag_list"], 4)),
            ("embeddings.feedid", _emb(V["feedid"], 16))]
    t = "transformer_blocks.0."
    mods += [(t + "position_embedding", nn.Embedding(51, 16))]
    mods += [(t + n, nn.Linear(16, 16)) for n in ("w_q", "w_k", "w_v", "w_o")]
    mods += [(t + "norm1", nn.LayerNorm(16)), (t + "norm2", nn.LayerNorm(16)), (t + "ffn.0", nn.Linear(16, 16)),
             (t + "ffn.3", nn.Linear(16, 16))]
    mods += [("dnn.0", nn.Linear(66, 512)), ("dnn.1", nn.BatchNorm1d(512)), ("dnn.4", nn.Linear(512, 256)),
             ("dnn.5", nn.BatchNorm1d(256)), ("dnn.8", nn.Linear(256, 128)), ("dnn.9", nn.BatchNorm1d(128)),
             ("dnn.12", nn.Linear(128, 1))]
    return mods


def _ref_afm():
    """afm.py:74-90 (embedding 8, attention factor 128)."""
    cols = ["userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list"]
    mods = [("dense_layer", nn.Linear(16, 1))] + [(f"embeddings.{c}", _emb(V[c], 8)) for c in cols]
    mods += [("attention.0", nn.Linear(8, 128)), ("attention.2", nn.Linear(128, 1)), ("p", nn.Linear(8, 1))]
    return mods


def _ref_deepcrossing():
    """deepcrossing.py:122-137."""
    mods = [("embeddings.userid", _emb(V["userid"], 16)), ("embeddings.device", _emb(V["device"], 2)),
            ("embeddings.authorid", _emb(V["authorid"], 4)), ("embeddings.bgm_song_id", _emb(V["bgm_song_id"], 4)),
            ("embeddings.bgm_singer_id", _emb(V["bgm_singer_id"], 4)),
            ("embeddings.manual_tag_list", _emb(V["manual_tag_list"], 4))]
    return mods + [("output_layer", nn.Linear(50, 1))]


def _rankops(name):
    if name == "dcn":
        return rankops.DCNModel(None, vocab_sizes=V)
    if name == "deepfm":
        return rankops.DeepFM(None, vocab_sizes={f: V[f] for f in rankops.deepfm.WECHAT_FIELDS})
    if name == "din":
        return rankops.DIN(None, vocab_sizes=V)
    if name == "bst":
        return rankops.BSTModel(None, vocab_sizes=V)
    if name == "afm":
        return rankops.AFM(H.afm_feature_columns(V), 8, 128)
    if name == "deepcrossing":
        return rankops.DeepCrossingModel(None, vocab_sizes=V)


REF = {"dcn": _ref_dcn, "deepfm": _ref_deepfm, "din": _ref_din, "bst": _ref_bst, "afm": _ref_afm,
       "deepcrossing": _ref_deepcrossing}


def test_seeded_construction_matches_reference_order():
    for name, make_ref in REF.items():
        torch.manual_seed(1234)
        expected = {}
        for prefix, mod in make_ref():
            for k, v in mod.state_dict().items():
                expected[f"{prefix}.{k}"] = v
        torch.manual_seed(1234)
        got = _rankops(name).state_dict()
        # every reference parameter/buffer exists with the same value (rankops adds no keys)
        assert set(got) == set(expected) | {k for k in got if k.startswith("fcn.") and (".alpha" in k or ".bn." in k
                                                                                           or k.split(".")[1] in ("2", "6", "10"))}, name
        for k, v in expected.items():
            assert torch.equal(got[k], v), f"{name}: {k}"


def test_din_state_dict_has_dice_and_bn_keys():
    keys = set(_rankops("din").state_dict())
    for i in (1, 5, 9):
        assert {f"fcn.{i}.alpha", f"fcn.{i}.bn.running_mean", f"fcn.{i}.bn.running_var"} <= keys
    for i in (2, 6, 10):
        assert {f"fcn.{i}.weight", f"fcn.{i}.bias", f"fcn.{i}.running_mean"} <= keys


def test_dcn_has_no_cross_keys_and_loads_reference_checkpoint_layout():
    m = _rankops("dcn")
    sd = m.state_dict()
    assert not any("cross" in k for k in sd)
    assert len(sd) == 14  # the reference checkpoint holds 14 tensors
    m.load_state_dict({k: torch.randn_like(v) for k, v in sd.items()}, strict=True)


def test_constructor_signatures_mirror_reference():
    sig = inspect.signature(rankops.DCNModel.__init__)
    assert list(sig.parameters)[:4] == ["self", "vocab_dir", "hidden_units", "num_cross_layer"]
    sig = inspect.signature(rankops.DIN.__init__)
    assert list(sig.parameters)[:9] == ["self", "vocab_dir", "hidden_units", "activation", "dropout_rate",
                                        "batch_norm", "use_softmax", "l2_lambda", "mini_batch_aware_regularization"]
    sig = inspect.signature(rankops.BSTModel.__init__)
    assert list(sig.parameters)[:11] == ["self", "vocab_dir", "hidden_units", "dropout_rate", "batch_norm", "d_model",
                                         "nhead", "num_transformer_blocks", "max_seq_length", "pooling_method",
                                         "vocab_sizes"]
    assert list(inspect.signature(rankops.DIN.forward).parameters) == ["self", "dense", "category", "sequence",
                                                                        "target"]
    assert list(inspect.signature(rankops.BSTModel.forward).parameters) == ["self", "dense", "category",
                                                                             "seq_feedid", "seq_length"]


def test_vocabulary_files_set_table_rows(tmp_path):
    """Table rows = len(vocab file lines) + 1; a missing file counts as empty (dcn.py:118-126,154-159)."""
    for f, n in (("userid.txt", 5), ("device.txt", 2), ("authorid.txt", 3), ("bgm_song_id.txt", 4),
                 ("bgm_singer_id.txt", 1), ("manual_tag_id.txt", 7)):
        (tmp_path / f).write_text("".join(f"{f}_{i}\n" for i in range(n)))
    m = rankops.DCNModel(str(tmp_path))
    assert m.embeddings["userid"].num_embeddings == 6
    assert m.embeddings["manual_tag_list"].num_embeddings == 8
    assert m.vocab_sizes["feedid"] == 1  # feedid.txt missing
    cols, labels = rankops.create_feature_columns(str(tmp_path))
    assert labels == ["read_comment"] and len(cols["vocab"]["manual_tag_list"]) == 7
    assert cols["vocab"]["feedid"] == []


def test_fused_mlp_envelope():
    assert common.fused_mlp_fits(960, [512, 256, 128])
    assert common.fused_mlp_fits(50, [128, 50, 128, 50])
    assert not common.fused_mlp_fits(50, [1024])
    assert not common.fused_mlp_fits(2000, [64])


def test_interaction_weight_modes():
    calls = []

    def draw():  # an H2Spec whose fill counts its draws
        def fill(v):
            calls.append(1)
            v[0].normal_()
        return common.H2Spec([(3,)], fill, lambda v: v[0])

    iw = common.InteractionWeights("frozen", draw)
    a = iw.get("cpu")
    b = iw.get("cpu")
    assert a is b and len(calls) == 1
    iw = common.InteractionWeights("per_call", draw)
    iw.get("cpu")
    iw.get("cpu")
    assert len(calls) == 3
    try:
        common.InteractionWeights("bogus", draw)
    except ValueError:
        pass
    else:
        raise AssertionError


def test_package_layout():
    assert os.path.isdir(os.path.join(H.PKG_DIR, "csrc"))
    assert os.path.isfile(os.path.join(H.REPO, "include", "rankops.h"))


def test_h2_spec_draws_equal_module_construction():
    """The per-call H2 draws (common.*_spec: the reference's generator calls into preallocated
    tensors, which the GPU path makes straight into a pinned staging buffer) are bit-identical to
    constructing the reference's layers: din_attention's three nn.Linear (din.py:61-67),
    cross_layer's xavier_normal_ / zeros_ (dcn.py:37-41), residual_unit's two nn.Linear
    (deepcrossing.py:37-39)."""
    import math
    import torch.nn as nn
    from rankops import common
    torch.manual_seed(11)
    mods = [nn.Linear(4 * 16, 64), nn.Linear(64, 32), nn.Linear(32, 1)]
    want = [t.detach() for m in mods for t in (m.weight, m.bias)]
    torch.manual_seed(11)
    got = common.draw_din_attention(16)
    assert all(torch.equal(a, b) for a, b in zip(want, got))
    torch.manual_seed(12)
    ws, bs = [], []
    for _ in range(2):
        w, b = torch.zeros(50, 1), torch.zeros(50, 1)
        nn.init.xavier_normal_(w)
        nn.init.zeros_(b)
        ws.append(w.reshape(50))
        bs.append(b.reshape(50))
    torch.manual_seed(12)
    W, B = common.draw_cross_layers(50, 2)
    assert torch.equal(W, torch.stack(ws)) and torch.equal(B, torch.stack(bs))
    torch.manual_seed(13)
    units = []
    for _ in range(3):
        a, b = nn.Linear(50, 128), nn.Linear(128, 50)
        units.append([t.detach() for t in (a.weight, a.bias, b.weight, b.bias)])
    torch.manual_seed(13)
    got = common.draw_residual_units(50, 128, 3)
    assert all(torch.equal(x, y) for u, v in zip(units, got) for x, y in zip(u, v))
    assert math.isclose(float(torch.empty(0).numel()), 0.0)
