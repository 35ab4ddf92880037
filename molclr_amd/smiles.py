"""SMILES featuriser for the binary graph shards.

The reference featurises each molecule with RDKit (``Chem.MolFromSmiles``,
dataset/dataset.py:61-109); RDKit is not installed in this image, so this
module parses SMILES itself and emits the reference's features:

* ``x[i] = [ATOM_LIST.index(Z), CHIRALITY_LIST.index(tag)]``: type index Z-1;
  chirality 0 none, 1 CW (``@@`` / ``@TH2``), 2 CCW (``@`` / ``@TH1``),
  3 other (``@AL``, ``@SP``, ``@TB``, ``@OH`` forms);
* one bond per RDKit bond, expanded to the directed pair (s,e),(e,s) with
  ``[BOND_LIST.index(type), BONDDIR_LIST.index(dir)]`` (dataset.py:93-109).

RDKit conventions restated (rdkit is unpinned in README.md:40, so this is
**parity unpinned**; the tests pin hand-derived cases):

* atoms are numbered in SMILES order; explicit ``[H]`` atoms bonded to a heavy
  atom are removed (MolFromSmiles' RemoveHs);
* chain bonds are numbered in parse order and ring-closure bonds after all of
  them, by ring-closure number, then appearance (RDKit's CloseMolRings over
  its bookmark map), begin atom = the atom that opened the ring;
* an unmarked bond between two aromatic atoms is AROMATIC if it lies on a
  ring, else SINGLE (sanitisation cannot leave a chain bond aromatic); ``:``
  is AROMATIC; ``/`` and ``\\`` are SINGLE with ENDUPRIGHT / ENDDOWNRIGHT,
  kept only on bonds next to a double bond (the stereo cleanup clears the
  others).

``featurise(..., add_hs=True)`` is ``Chem.AddHs`` on top (the mixed
augmentation's input, dataset/dataset_mix.py:87-88), with RDKit's
implicit-hydrogen rule for the organic subset (default valences B 3, C 4,
N 3, O 2, P 3/5, S 2/4/6, halogens 1; aromatic bonds count 1.5 and an aromatic
atom is capped at its first default valence) and the bracket H counts.

Not restated: aromaticity *perception* of Kekulé input (``C1=CC=CC=C1``
stays single/double; PubChem-10M-clean is RDKit canonical, i.e. already
aromatic), and the removal of chirality tags from atoms that are not
stereocentres.  Inputs RDKit would reject or that fall outside the
reference's vocabulary (``*``, quadruple bonds, aromatic atoms off any ring,
unclosed rings) raise ValueError, where the reference would crash.
"""
from __future__ import annotations

import re

import numpy as np

_ELEMENTS = (
    "H He Li Be B C N O F Ne Na Mg Al Si P S Cl Ar K Ca Sc Ti V Cr Mn Fe Co Ni Cu Zn Ga Ge As "
    "Se Br Kr Rb Sr Y Zr Nb Mo Tc Ru Rh Pd Ag Cd In Sn Sb Te I Xe Cs Ba La Ce Pr Nd Pm Sm Eu "
    "Gd Tb Dy Ho Er Tm Yb Lu Hf Ta W Re Os Ir Pt Au Hg Tl Pb Bi Po At Rn Fr Ra Ac Th Pa U Np "
    "Pu Am Cm Bk Cf Es Fm Md No Lr Rf Db Sg Bh Hs Mt Ds Rg Cn Nh Fl Mc Lv Ts Og").split()
Z_OF = {s: i + 1 for i, s in enumerate(_ELEMENTS)}
_ORGANIC = ("Cl", "Br", "B", "C", "N", "O", "P", "S", "F", "I")
_AROMATIC_ORGANIC = ("b", "c", "n", "o", "p", "s")
_AROMATIC_BRACKET = {"se": 34, "as": 33, "te": 52, "si": 14, "b": 5, "c": 6, "n": 7, "o": 8,
                     "p": 15, "s": 16}

SINGLE, DOUBLE, TRIPLE, AROMATIC = 0, 1, 2, 3   # BOND_LIST (dataset.py:33-38)
DIR_NONE, DIR_UP, DIR_DOWN = 0, 1, 2            # BONDDIR_LIST (dataset.py:39-43)
CHI_NONE, CHI_CW, CHI_CCW, CHI_OTHER = 0, 1, 2, 3  # CHIRALITY_LIST (dataset.py:27-32)

_BRACKET = re.compile(r"\[(\d+)?([A-Z][a-z]?|se|as|te|si|[bcnops])"
                      r"(@(?:@|TH[12]|AL[12]|SP[123]|TB\d{1,2}|OH\d{1,2})?)?"
                      r"(H\d?)?([+-]+\d*)?(:\d+)?\]")
_BOND_SYM = {"-": (SINGLE, DIR_NONE), "=": (DOUBLE, DIR_NONE), "#": (TRIPLE, DIR_NONE),
             ":": (AROMATIC, DIR_NONE), "/": (SINGLE, DIR_UP), "\\": (SINGLE, DIR_DOWN)}


def _chirality(tag: str | None) -> int:
    if not tag:
        return CHI_NONE
    if tag in ("@", "@TH1"):
        return CHI_CCW
    if tag in ("@@", "@TH2"):
        return CHI_CW
    return CHI_OTHER


def parse(smiles: str):
    """Atoms [(Z, chirality, aromatic, is_plain_H, bracket H count or None)],
    bonds [(begin, end, type|None, dir)] (type None = unmarked) in RDKit bond
    order.  The H count is None for organic-subset atoms (implicit Hs)."""
    atoms, chain, ring_bonds = [], [], []
    open_rings = {}   # ring number -> (atom, bond symbol or None, order of opening)
    closures = []     # (ring number, opening order, begin, end, symbol)
    stack = []
    prev = None
    pending = None    # bond symbol waiting for the next atom
    i, n = 0, len(smiles)
    opened = 0
    while i < n:
        ch = smiles[i]
        if ch in _BOND_SYM:
            if pending is not None:
                raise ValueError(f"two bond symbols at {i}")
            pending = ch
            i += 1
            continue
        if ch == "$":
            raise ValueError("quadruple bond is outside BOND_LIST")
        if ch == "(":
            if prev is None:
                raise ValueError("branch before any atom")
            stack.append(prev)
            i += 1
            continue
        if ch == ")":
            if not stack:
                raise ValueError("unbalanced ')'")
            prev = stack.pop()
            i += 1
            continue
        if ch == ".":
            prev, pending = None, None
            i += 1
            continue
        if ch.isdigit() or ch == "%":
            if prev is None:
                raise ValueError("ring closure before any atom")
            if ch == "%":
                if smiles[i + 1:i + 2] == "(":
                    j = smiles.index(")", i)
                    num, i = int(smiles[i + 2:j]), j + 1
                else:
                    num, i = int(smiles[i + 1:i + 3]), i + 3
            else:
                num, i = int(ch), i + 1
            if num in open_rings:
                a, sym, order = open_rings.pop(num)
                if sym is not None and pending is not None and sym != pending:
                    raise ValueError(f"conflicting ring-closure bonds for ring {num}")
                closures.append((num, order, a, prev, sym if sym is not None else pending))
            else:
                open_rings[num] = (prev, pending, opened)
                opened += 1
            pending = None
            continue
        # an atom
        if ch == "[":
            m = _BRACKET.match(smiles, i)
            if not m:
                raise ValueError(f"unsupported bracket atom at {i}: {smiles[i:i + 12]!r}")
            iso, sym, chi, hs, _, _ = m.groups()
            arom = sym in _AROMATIC_BRACKET and sym.islower()
            Z = _AROMATIC_BRACKET[sym] if arom else Z_OF.get(sym)
            if Z is None:
                raise ValueError(f"unknown element {sym!r}")
            plain_h = Z == 1 and iso is None
            nh = 0 if not hs else (int(hs[1:]) if len(hs) > 1 else 1)
            atoms.append((Z, _chirality(chi), arom, plain_h, nh))
            i = m.end()
        elif ch == "*":
            raise ValueError("dummy atom '*' (atomic number 0) is outside ATOM_LIST")
        else:
            sym = next((s for s in _ORGANIC if smiles.startswith(s, i)), None)
            if sym is not None:
                atoms.append((Z_OF[sym], CHI_NONE, False, False, None))
                i += len(sym)
            elif ch in _AROMATIC_ORGANIC:
                atoms.append((Z_OF[ch.upper()], CHI_NONE, True, False, None))
                i += 1
            else:
                raise ValueError(f"unexpected character {ch!r} at {i}")
        cur = len(atoms) - 1
        if prev is not None:
            chain.append((prev, cur, pending))
        elif pending is not None:
            raise ValueError("bond symbol with nothing to bond to")
        prev, pending = cur, None
    if open_rings:
        raise ValueError(f"unclosed ring(s) {sorted(open_rings)}")
    if stack:
        raise ValueError("unbalanced '('")
    # ring closures after the chain bonds: by ring number, then order of opening
    for num, order, a, b, sym in sorted(closures, key=lambda c: (c[0], c[1])):
        ring_bonds.append((a, b, sym))
    bonds = []
    for a, b, sym in chain + ring_bonds:
        t, d = _BOND_SYM[sym] if sym is not None else (None, DIR_NONE)
        bonds.append((a, b, t, d))
    return atoms, bonds


def _ring_bonds(n_atoms: int, bonds) -> np.ndarray:
    """Bond k is on a ring iff it is not a bridge (Tarjan, iterative)."""
    adj = [[] for _ in range(n_atoms)]
    for k, (a, b, _, _) in enumerate(bonds):
        adj[a].append((b, k))
        adj[b].append((a, k))
    disc = [-1] * n_atoms
    low = [0] * n_atoms
    on_ring = np.ones(len(bonds), dtype=bool)
    t = 0
    for root in range(n_atoms):
        if disc[root] >= 0:
            continue
        disc[root] = low[root] = t
        t += 1
        it = [(root, -1, iter(adj[root]))]
        while it:
            v, pk, nbrs = it[-1]
            for w, k in nbrs:
                if k == pk:
                    continue
                if disc[w] < 0:
                    disc[w] = low[w] = t
                    t += 1
                    it.append((w, k, iter(adj[w])))
                    break
                low[v] = min(low[v], disc[w])
            else:
                it.pop()
                if it:
                    u = it[-1][0]
                    low[u] = min(low[u], low[v])
                    if low[v] > disc[u]:
                        on_ring[pk] = False
    return on_ring


# RDKit's default valences of the organic subset (implicit hydrogens)
_DEFAULT_VALENCE = {5: (3,), 6: (4,), 7: (3,), 8: (2,), 15: (3, 5), 16: (2, 4, 6), 9: (1,),
                    17: (1,), 35: (1,), 53: (1,)}
_BOND_ORDER = {SINGLE: 1.0, DOUBLE: 2.0, TRIPLE: 3.0, AROMATIC: 1.5}


def _implicit_hs(Z: int, aromatic: bool, valence: float) -> int:
    """RDKit's implicit-H count of an organic-subset atom: explicit valence
    with aromatic bonds at 1.5 (an aromatic atom above its first default
    valence is taken at it), rounded, then the smallest default valence that
    is not below it minus the valence.  Above every default valence RDKit
    rejects the molecule."""
    allowed = _DEFAULT_VALENCE.get(Z)
    if allowed is None:
        raise ValueError(f"element {Z} is not in the SMILES organic subset")
    if aromatic and valence > allowed[0]:
        valence = float(allowed[0])
    v = int(valence + 0.1 + 0.5)   # round(valence + 0.1), half up
    for a in allowed:
        if a >= v:
            return a - v
    raise ValueError(f"explicit valence {v} of element {Z} exceeds its default valences")


def featurise(smiles: str, add_hs: bool = False):
    """A dataset.Molecule (x [N,2], edge_index [2,2M], edge_attr [2M,2],
    numpy int64) with the reference's features (dataset.py:65-109).

    ``add_hs`` adds the hydrogens explicitly, as ``Chem.AddHs(mol)`` does for
    the mixed augmentation (dataset/dataset_mix.py:87-88): after the heavy
    atoms, for every atom in order, its hydrogens (bracket count, implicit
    count of an organic-subset atom, and the explicit ``[H]`` atoms that
    RemoveHs folded into it) each become an atom [0, 0] (ATOM_LIST.index(1),
    CHI_UNSPECIFIED) bonded to it by a SINGLE bond, direction NONE, begin atom
    the heavy one, appended after the original bonds."""
    from .dataset import Molecule
    atoms, bonds = parse(smiles)
    # RemoveHs: drop plain [H] atoms that hang off another atom
    deg = np.zeros(len(atoms), dtype=np.int64)
    for a, b, _, _ in bonds:
        deg[a] += 1
        deg[b] += 1
    keep = [not (at[3] and deg[k] > 0) for k, at in enumerate(atoms)]
    remap = np.cumsum(keep) - 1
    folded = np.zeros(len(atoms), dtype=np.int64)   # removed [H] per surviving atom
    for a, b, _, _ in bonds:
        if keep[a] and not keep[b]:
            folded[a] += 1
        if keep[b] and not keep[a]:
            folded[b] += 1
    kept_atoms = [at for k, at in enumerate(atoms) if keep[k]]
    folded = folded[np.asarray(keep, dtype=bool)]
    kept_bonds = [(int(remap[a]), int(remap[b]), t, d) for a, b, t, d in bonds
                  if keep[a] and keep[b]]
    if not kept_atoms:
        raise ValueError("no atoms")
    on_ring = _ring_bonds(len(kept_atoms), kept_bonds)
    arom = [at[2] for at in kept_atoms]
    for k, at in enumerate(kept_atoms):
        if at[2] and not any(on_ring[j] for j, (a, b, _, _) in enumerate(kept_bonds) if k in (a, b)):
            raise ValueError("aromatic atom outside any ring (RDKit rejects it)")
    types = []
    for k, (a, b, t, d) in enumerate(kept_bonds):
        if t is None:
            t = AROMATIC if (arom[a] and arom[b] and on_ring[k]) else SINGLE
        types.append(t)
    # directional flags survive only next to a double bond
    dbl_atoms = {x for (a, b, _, _), t in zip(kept_bonds, types) if t == DOUBLE for x in (a, b)}
    dirs = [d if (types[k] == SINGLE and (a in dbl_atoms or b in dbl_atoms)) else DIR_NONE
            for k, (a, b, _, d) in enumerate(kept_bonds)]
    xs = [[Z - 1, chi] for Z, chi, *_ in kept_atoms]
    edges = [(a, b, types[k], dirs[k]) for k, (a, b, _, _) in enumerate(kept_bonds)]
    if add_hs:
        valence = np.zeros(len(kept_atoms))
        for (a, b, _, _), t in zip(kept_bonds, types):
            valence[a] += _BOND_ORDER[t]
            valence[b] += _BOND_ORDER[t]
        valence += folded  # the folded [H] atoms were single bonds
        for k, (Z, _, ar, _, nh) in enumerate(kept_atoms):
            h = (nh if nh is not None else _implicit_hs(Z, ar, valence[k])) + int(folded[k])
            for _ in range(h):
                xs.append([0, CHI_NONE])
                edges.append((k, len(xs) - 1, SINGLE, DIR_NONE))
    x = np.array(xs, dtype=np.int64).reshape(-1, 2)
    M = len(edges)
    ei = np.empty((2, 2 * M), dtype=np.int64)
    ea = np.empty((2 * M, 2), dtype=np.int64)
    for k, (a, b, t, d) in enumerate(edges):
        ei[:, 2 * k] = (a, b)
        ei[:, 2 * k + 1] = (b, a)
        ea[2 * k] = ea[2 * k + 1] = (t, d)
    return Molecule(x, ei, ea)
