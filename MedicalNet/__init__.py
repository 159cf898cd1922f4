"""MedicalNet API shim (MedicalNet.model.generate_model, MedicalNet.setting.parse_opts)."""
