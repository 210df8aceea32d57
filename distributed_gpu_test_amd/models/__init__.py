from .simple_net import SimpleNet, pack_simple_net, simple_net_layout, simple_net_numel  # noqa: F401
