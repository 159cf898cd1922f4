"""Import-path shim: ``pkg.*`` module paths of the reference resolve to the MI355X drop-ins
in multimodal_alzheimer_amd, so unchanged reference drivers (train_*.py, pkg/inference/*)
pick them up."""
