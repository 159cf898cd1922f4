"""The reference's TabPFN fusion chain on the drop-in surface, CPU only (no kernels run):
Tabular_MRT_Model / PET_TABULAR_CNN (stage 2) and All_Modalities_Fusion (stage 3) built
through PL checkpoint files as all_modalities_fusion.py:17-31 builds them.

  * state_dict keys identical to the real reference classes' (fixture
    all_modalities_fusion, tests/golden/make_golden.py), for the unfrozen build and the
    default (frozen) build, and the same parameters left trainable by the freeze
    (all_modalities_fusion.py:34-47 + the stage-2 freezes);
  * the cut: each stage-2 ``model_fuse`` is its stage2out alone (:29-31);
  * without TabPFN and without a registered backend the tabular models fail loudly;
  * get_avg_activation restates dl_approach.py:71-78.
"""
import numpy as np
import pytest
import torch

import multimodal_alzheimer_amd as M
from multimodal_alzheimer_amd import tabular
from tests import _golden as G


@pytest.fixture(autouse=True)
def _clear_backend():
    yield
    tabular.set_backend(None)


@pytest.mark.parametrize("lr_pretrained", [1e-5, None])
def test_chain_state_dict_and_freeze_match_reference(tmp_path, lr_pretrained):
    g = G.load("all_modalities_fusion")
    m = G.amf_checkpoint_chain(str(tmp_path), lr_pretrained=lr_pretrained)
    keys = list(m.state_dict().keys())
    if lr_pretrained:
        assert keys == list(g["state_dict_keys"])
        assert all(p.requires_grad for p in m.parameters())
    else:
        assert keys == list(g["frozen_state_dict_keys"])
        trainable = [n for n, p in m.named_parameters() if p.requires_grad]
        assert trainable == list(g["frozen_trainable"])
    for sub in (m.model_anat_pet, m.model_anat_tab, m.model_pet_tab):
        assert len(sub.model_fuse) == 1 and sub.model_fuse[0] is sub.stage2out


def test_optimizer_groups(tmp_path):
    """all_modalities_fusion.py:98-137: the stage-3 head at lr; with lr_pretrained the
    stage-1/2 parts at lr_pretrained (the TabPFN transformers' parameters included)."""
    m = G.amf_checkpoint_chain(str(tmp_path), lr_pretrained=1e-5)
    opt = m.configure_optimizers()
    lrs = sorted({g["lr"] for g in opt.param_groups})
    assert lrs == [1e-5, 1e-3]
    head = {id(p) for p in m.model_fuse.parameters()}
    for grp in opt.param_groups:
        ids = {id(p) for p in grp["params"]}
        assert (ids <= head) == (grp["lr"] == 1e-3)
    n_opt = sum(len(g["params"]) for g in opt.param_groups)
    tab = sum(len(list(x.model_tabular.model[2].parameters()))
              for x in (m.model_anat_tab, m.model_pet_tab))
    assert n_opt == len(list(m.model_fuse.parameters())) + tab + sum(
        len(list(x.parameters())) for x in (
            m.model_anat_pet.model_pet, m.model_anat_pet.model_mri, m.model_anat_pet.stage2out,
            m.model_anat_pet.reduce_dim_mri, m.model_pet_tab.model_pet,
            m.model_pet_tab.stage2out, m.model_pet_tab.reduce_tab, m.model_anat_tab.model_mri,
            m.model_anat_tab.stage2out, m.model_anat_tab.reduce_tab))


def test_tabpfn_missing_fails_loudly(tmp_path):
    tabular.set_backend(None)
    try:
        import tabpfn  # noqa: F401
        pytest.skip("tabpfn is installed")
    except ImportError:
        pass
    p = str(tmp_path / "mri.ckpt")
    M.Anat_CNN(G.anat_hparams(10)).save_checkpoint(p)
    with pytest.raises(tabular.TabPFNUnavailable, match="tabpfn"):
        M.Tabular_MRT_Model(G.anat_hparams(10, ensemble_size=4), path_mri=p)


def test_get_avg_activation():
    """dl_approach.py:71-78 on a known tensor: the test rows, averaged over members."""
    acts = torch.arange(5 * 3 * 4, dtype=torch.float32).reshape(5, 3, 4)
    out = tabular.get_avg_activation(acts, 3, 2)
    np.testing.assert_array_equal(out.numpy(), acts[2:].mean(1).numpy())
    assert out.shape == (3, 4)


def test_tri_resnet_tabular_keys_match_oracle_fixture():
    """config 5's network (Tri_ResNet_Tabular_Fusion) has the state_dict of the oracle
    restatement its full-size fixture (tri_160) was generated from"""
    g = G.load("tri_160")
    m = M.Tri_ResNet_Tabular_Fusion(G.anat_hparams(10, fl_gamma=2, resnet_depth_mri=34,
                                                   resnet_depth_pet=18))
    assert list(m.state_dict().keys()) == list(g["state_dict_keys"])
