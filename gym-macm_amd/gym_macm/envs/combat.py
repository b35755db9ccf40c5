"""cm-tdm-v0 / cm-ctdm-v0 (reference gym_macm/envs/combat.py).

Not built in this version. The reference classes cannot be constructed as
shipped (combat.py:65 uses `combatSettings`, which combat.py:8 never imports), so
their semantics must first be decided; TDM is the next
row of the hot-path scope table. Constructing them
raises with that explanation instead of silently falling back to anything.
"""


class TDM(object):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(
            "cm-tdm-v0 is not built yet (the reference's TDM raises NameError at combat.py:65); "
            "see DESIGN.md 'Out of scope / next'")


class ControlledTDM(TDM):
    pass
