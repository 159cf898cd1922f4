"""CPU oracle for the MI355X 3D-volume training hot path -- TEST INFRASTRUCTURE ONLY.

Nothing in ``multimodal_alzheimer_amd/`` imports this package.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it, and only
as the checker / CPU baseline, never as the thing measured or shipped.

Contents
--------
* ``prng``            -- counter-based splitmix64 generator; regenerates weights and
                         volumes bit-identically on any host (fixtures store only seeds
                         and outputs).
* ``medicalnet_ref``  -- torch-CPU restatement of the third-party Tencent/MedicalNet
                         3D-ResNet (BasicBlock/Bottleneck, shortcut "B", dilated
                         layer3/layer4) that the reference imports at
                         ``pkg/models/mri_models/anat_cnn.py:4-5`` but does not vendor.
* ``models_ref``      -- torch-CPU restatement of the reference heads, fusion wiring,
                         ``general_step`` precision contract and the focal /
                         weighted-CE losses (file:line citations on every function).

Parity pinning
--------------
``models_ref`` is pinned against golden vectors produced by importing the *real*
reference ``pkg`` code in the build container (``tests/golden/make_golden.py``).
MedicalNet itself is absent offline and unpinned by any reference test: the ResNet
arithmetic is pinned against "reference pkg code + this restatement" only
 -- "parity unpinned against genuine MedicalNet".
"""
