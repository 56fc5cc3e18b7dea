"""CPU oracle for the voxel-graph GAN hot path -- TEST INFRASTRUCTURE ONLY.

Nothing in the product package (``building-gan-...-_amd/vgan``) imports this
package.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker / the timed CPU baseline.

Contents
--------
``pyg``        restatement of the torch-geometric 2.6.1 operators the reference
               calls (GATConv heads=1, utils.softmax index path, GraphNorm with
               batch=None, Sequential, Batch) -- the arithmetic of the path.
``dense``      an independent dense-adjacency derivation of the same operators
               (masked N x N softmax), used to cross-check ``pyg``.
``reference``  restatement of the reference models (``models.py:14-245``) and of
               the trainer step (``trainer.py:291-502``) on top of ``pyg``.
``shim``       a ``sys.modules`` shim that lets the *reference's own* ``models.py``
               / ``trainer.py`` import in this container against ``pyg``; used
               only by ``tests/golden/make_golden.py`` to produce fixtures.

Parity status (see DESIGN.md "Oracle"): the reference's orchestration
(type-mean, concatenation order, Gumbel straight-through, losses, gradient
penalty, Adam step) is pinned by fixtures produced by executing the reference
``models.py``/``trainer.py`` here.  The torch-geometric operator semantics are
restated from the published 2.6.1 source (the package is absent and not
installable offline) and cross-checked against ``dense`` -- that layer is
"parity unpinned" against PyG itself.
"""
