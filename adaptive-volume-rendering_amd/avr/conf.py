"""Minimal stand-in for a pyhocon ConfigTree (pyhocon is not installed here).

`from_conf(conf)` in the reference reads `conf.get_int/get_float/get_bool/
get_string(key, default)` and `conf["sub"]`; any mapping wrapped in Conf
supports the same calls, and a real pyhocon ConfigTree works unchanged.
"""


class Conf(dict):
    def _get(self, key, default):
        cur = self
        for part in key.split("."):
            if not isinstance(cur, dict) or part not in cur:
                return default
            cur = dict.__getitem__(cur, part)
        return cur

    def get_int(self, key, default=None):
        v = self._get(key, default)
        return None if v is None else int(v)

    def get_float(self, key, default=None):
        v = self._get(key, default)
        return None if v is None else float(v)

    def get_bool(self, key, default=None):
        v = self._get(key, default)
        if isinstance(v, str):
            return v.strip().lower() in ("1", "true", "yes", "on")
        return None if v is None else bool(v)

    def get_string(self, key, default=None):
        v = self._get(key, default)
        return None if v is None else str(v)

    def get_config(self, key, default=None):
        v = self._get(key, default)
        return Conf(v) if isinstance(v, dict) else v

    def __getitem__(self, key):
        v = dict.__getitem__(self, key)
        return Conf(v) if isinstance(v, dict) and not isinstance(v, Conf) else v


# conf/default.conf (model{}, normal_renderer{}, raymarcher{}, adaptive_renderer{}) restated as data.
DEFAULT_MODEL = {
    "use_encoder": True, "use_global_encoder": False, "use_xyz": True, "canon_xyz": False, "use_code": True,
    "code": {"num_freqs": 6, "freq_factor": 1.5, "include_input": True},
    "use_viewdirs": True, "use_code_viewdirs": False,
    "mlp_coarse": {"type": "resnet", "n_blocks": 3, "d_hidden": 512},
    "mlp_fine": {"type": "resnet", "n_blocks": 3, "d_hidden": 512},
    "encoder": {"backbone": "resnet34", "pretrained": True, "num_layers": 4},
}
DEFAULT_NORMAL_RENDERER = {"near": 0.8, "far": 1.8, "n_coarse": 64, "n_fine": 32, "n_fine_depth": 16,
                           "depth_std": 0.01, "white_back": True}
DEFAULT_RAYMARCHER = {"num_feature_channels": 512, "raymarch_steps": 10}
DEFAULT_ADAPTIVE_RENDERER = {"num_feature_channels": 512, "raymarch_steps": 10, "epsilon": 0.15, "n_coarse": 20,
                             "white_back": True}
# conf/default_mv.conf overrides (5 blocks, combine after the 3rd)
DEFAULT_MV_MLP = {"type": "resnet", "n_blocks": 5, "d_hidden": 512, "combine_layer": 3, "combine_type": "average"}


def default_conf(multiview=False):
    import copy
    model = copy.deepcopy(DEFAULT_MODEL)
    if multiview:
        model["mlp_coarse"] = dict(DEFAULT_MV_MLP)
        model["mlp_fine"] = dict(DEFAULT_MV_MLP)
    return Conf({"model": model, "normal_renderer": dict(DEFAULT_NORMAL_RENDERER),
                 "raymarcher": dict(DEFAULT_RAYMARCHER), "adaptive_renderer": dict(DEFAULT_ADAPTIVE_RENDERER)})
