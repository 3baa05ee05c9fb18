"""lss_carla_amd -- MI355X-native Lift-Splat hot path behind the LiftSplatShoot surface.

Drop-in for ``src.models`` of shdragron/LSS-Carla: ``compile_model``,
``LiftSplatShoot`` (same ctor dicts, same ``forward(x, rots, trans, intrins,
post_rots, post_trans)``, same state_dict keys). The lift, geometry and splat
run as hand-written gfx950 HIP kernels in ``liblss_hip.so`` (C ABI declared in
``include/lss_hip.h``); the conv stacks are stock PyTorch-ROCm modules.

Heavy submodules are imported lazily so that host-only tools (synthetic inputs,
the ABI loader) work without a GPU.
"""
__version__ = "0.1.0"

_LAZY = {
    "compile_model": "models", "LiftSplatShoot": "models", "CamEncode": "models",
    "BevEncode": "models", "Up": "models",
    "gen_dx_bx": "tools", "SimpleLoss": "tools", "get_batch_iou": "tools", "get_batch_iou_device": "tools",
    "get_val_info": "tools", "QuickCumsum": "tools", "cumsum_trick": "tools",
}


def __getattr__(name):
    if name in _LAZY:
        import importlib
        mod = importlib.import_module(f"{__name__}.{_LAZY[name]}")
        return getattr(mod, name)
    raise AttributeError(name)
