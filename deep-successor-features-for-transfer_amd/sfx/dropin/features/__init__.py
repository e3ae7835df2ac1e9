"""sfx's SF library modules under the reference's package name ``features``.

After ``sfx.dropin.install()`` the top-level package ``features`` is this directory followed by
the user's own ``features`` directory: ``features.deep``, ``features.deep_sequential``,
``features.deep_sequential_tsf``, ``features.deep_phi`` and ``features.successor`` are sfx's, any
other module (``features.tabular``, ``features.deep_tsf_phi`` ...) is the user's."""
