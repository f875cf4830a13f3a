"""Deterministic synthetic clinical data (no datasets are reachable offline).

* :func:`synthetic_kb` -- TCM knowledge-base rows with the column schema of the
  reference's ``default_data`` CSVs (``matrice_plante_syndrome.csv``:
  nom_syndrome, nom_latin, nom_chinois, score_role; ``base_connaissance_tcm.csv``:
  nom_syndrome, nom_link, nom_latin, role_formule, score_role, description, ...), so the
  same CSV->sentence templating (semantic-indexer/indexer.py:50-94) applies.
* :func:`synthetic_notes` -- French clinical notes with realistic PII (names, dates,
  phones, e-mails, cities, nationalities) for the ingest -> deid -> index pipeline.
* :func:`synthetic_questions` -- practitioner questions drawn from a small template x
  syndrome x symptom grid (~470 distinct strings: the cache-hot "repeat" workload).
* :func:`synthetic_unique_questions` -- pairwise-distinct questions (the default QA
  benchmark workload: every request is new).
"""
from __future__ import annotations

import random

FIRST = ["Jean", "Marie", "Pierre", "Sophie", "Luc", "Claire", "Ahmed", "Fatima", "Yassine",
         "Camille", "Nicolas", "Julie", "Karim", "Emma", "Thomas", "Léa", "Hugo", "Chloé",
         "Mohamed", "Sarah", "Antoine", "Inès", "Louis", "Manon", "Omar", "Zoé", "Paul", "Lina"]
LAST = ["Martin", "Bernard", "Dubois", "Thomas", "Robert", "Richard", "Petit", "Durand",
        "Leroy", "Moreau", "Simon", "Laurent", "Lefebvre", "Michel", "Garcia", "Benali",
        "Haddad", "Roux", "Fournier", "Girard", "Bonnet", "Dupont", "Lambert", "Fontaine"]
CITIES = ["Paris", "Lyon", "Marseille", "Toulouse", "Casablanca", "Rabat", "Lille", "Nantes",
          "Bordeaux", "Montréal", "Genève", "Bruxelles", "Strasbourg", "Nice", "Fès"]
NATIONALITIES = ["française", "marocaine", "algérienne", "belge", "suisse", "canadienne",
                 "tunisienne", "sénégalaise"]
SYNDROMES = [
    "Vide de Qi de la Rate", "Stagnation du Qi du Foie", "Vide de Yin du Rein",
    "Vide de Yang du Rein", "Vide de Sang du Cœur", "Stase de Sang", "Chaleur-Humidité",
    "Glaires-Humidité", "Montée du Yang du Foie", "Vide de Qi du Poumon", "Froid-Vent",
    "Chaleur du Poumon", "Vide de Yin du Poumon", "Feu du Cœur", "Vide de Sang du Foie",
    "Humidité de la Rate", "Insomnie par vide du Cœur", "Vide de Jing", "Chaleur du Sang",
    "Stagnation alimentaire", "absence de transpiration", "fatigue chronique",
    "douleurs lombaires", "troubles menstruels", "céphalées", "vertiges", "toux sèche",
]
PLANTS = [
    ("Angelica sinensis", "当归", "Dang Gui"), ("Astragalus membranaceus", "黄芪", "Huang Qi"),
    ("Panax ginseng", "人参", "Ren Shen"), ("Glycyrrhiza uralensis", "甘草", "Gan Cao"),
    ("Atractylodes macrocephala", "白术", "Bai Zhu"), ("Poria cocos", "茯苓", "Fu Ling"),
    ("Rehmannia glutinosa", "地黄", "Di Huang"), ("Paeonia lactiflora", "白芍", "Bai Shao"),
    ("Ligusticum chuanxiong", "川芎", "Chuan Xiong"), ("Bupleurum chinense", "柴胡", "Chai Hu"),
    ("Ziziphus jujuba", "酸枣仁", "Suan Zao Ren"), ("Cordyceps sinensis", "冬虫夏草", "Dong Chong Xia Cao"),
    ("Lycium barbarum", "枸杞子", "Gou Qi Zi"), ("Schisandra chinensis", "五味子", "Wu Wei Zi"),
    ("Dimocarpus longan", "龙眼肉", "Long Yan Rou"), ("Polygala tenuifolia", "远志", "Yuan Zhi"),
    ("Cinnamomum cassia", "肉桂", "Rou Gui"), ("Zingiber officinale", "生姜", "Sheng Jiang"),
    ("Coptis chinensis", "黄连", "Huang Lian"), ("Scutellaria baicalensis", "黄芩", "Huang Qin"),
    ("Salvia miltiorrhiza", "丹参", "Dan Shen"), ("Codonopsis pilosula", "党参", "Dang Shen"),
    ("Dioscorea opposita", "山药", "Shan Yao"), ("Cornus officinalis", "山茱萸", "Shan Zhu Yu"),
]
ROLES = [("Empereur", 10), ("Ministre", 7), ("Assistant", 5), ("Messager", 3)]
ORGANS = ["Foie", "Rate", "Rein", "Cœur", "Poumon", "Estomac"]
MEDS = ["warfarine 5 mg", "apixaban 5 mg", "metformine 850 mg", "amlodipine 5 mg",
        "paracétamol 1 g", "oméprazole 20 mg", "lévothyroxine 75 µg", "atorvastatine 20 mg",
        "bisoprolol 2,5 mg", "ramipril 5 mg"]
SYMPTOMS = ["fatigue persistante", "insomnie", "sueurs nocturnes", "vertiges", "palpitations",
            "douleurs abdominales", "ballonnements", "toux sèche", "céphalées frontales",
            "frilosité", "irritabilité", "perte d'appétit", "douleurs lombaires",
            "bouffées de chaleur", "essoufflement à l'effort"]


def _rng(seed: int) -> random.Random:
    return random.Random(seed)


def synthetic_kb(n_matrix: int = 298, n_base: int = 349, seed: int = 0):
    """Returns (matrix_rows, base_rows) as lists of dicts with the reference CSV columns."""
    r = _rng(seed)
    matrix, base = [], []
    for _ in range(n_matrix):
        lat, zh, _pin = r.choice(PLANTS)
        matrix.append({"nom_syndrome": r.choice(SYNDROMES), "nom_latin": lat, "nom_chinois": zh,
                       "score_role": str(r.choice([3, 4, 5, 7, 9, 10, 11, 14, 20]))})
    for i in range(n_base):
        lat, zh, pin = r.choice(PLANTS)
        role, score = r.choice(ROLES)
        syn = r.choice(SYNDROMES)
        base.append({
            "id_syndrome": str(i + 1), "nom_syndrome": syn, "categorie_synd": r.choice(SYNDROMES[:8]),
            "organe_associe": r.choice(ORGANS), "nom_link": pin, "nom_latin": lat,
            "nom_chinois": zh, "role_formule": role, "score_role": str(score),
            "description": f"{r.choice(['Tonifie', 'Harmonise', 'Disperse', 'Rafraîchit', 'Nourrit'])} "
                           f"le {r.choice(['Qi', 'Sang', 'Yin', 'Yang', 'Jing'])} du {r.choice(ORGANS)}. "
                           f"Utilisée en cas de {r.choice(SYMPTOMS)} et de {r.choice(SYMPTOMS)}.",
        })
    return matrix, base


def _date(r: random.Random) -> str:
    return f"{r.randint(1, 28):02d}/{r.randint(1, 12):02d}/{r.randint(2015, 2025)}"


def _phone(r: random.Random) -> str:
    return "0" + str(r.randint(1, 7)) + " " + " ".join(f"{r.randint(0, 99):02d}" for _ in range(4))


def synthetic_note(i: int, seed: int = 0) -> dict:
    r = _rng(seed * 1_000_003 + i)
    fn, ln = r.choice(FIRST), r.choice(LAST)
    doc = f"Dr {r.choice(FIRST)} {r.choice(LAST)}"
    syn = r.choice(SYNDROMES)
    plants = r.sample(PLANTS, 3)
    sym = r.sample(SYMPTOMS, 3)
    email = f"{fn.lower()}.{ln.lower()}{r.randint(1, 99)}@example.com".replace("é", "e").replace("ï", "i")
    paras = [
        f"Compte-rendu de consultation du {_date(r)}.",
        f"Patient : {fn} {ln}, né le {_date(r)} à {r.choice(CITIES)}, nationalité {r.choice(NATIONALITIES)}. "
        f"Téléphone : {_phone(r)}. Courriel : {email}.",
        f"Motif : {sym[0]}, {sym[1]} et {sym[2]} depuis {r.randint(2, 30)} semaines.",
        f"Antécédents : traitement par {r.choice(MEDS)} ; suivi par {doc} à {r.choice(CITIES)}.",
        f"Examen : langue {r.choice(['pâle', 'rouge', 'enduit blanc', 'enduit jaune'])}, pouls "
        f"{r.choice(['fin', 'rapide', 'tendu', 'faible', 'glissant'])}. Tension {r.randint(100, 160)}/{r.randint(60, 95)} mmHg.",
        f"Bilan énergétique : syndrome « {syn} » avec atteinte du {r.choice(ORGANS)}.",
        "Prescription : " + ", ".join(f"{p[0]} ({p[1]}) {r.randint(3, 15)} g" for p in plants) +
        f", en décoction deux fois par jour pendant {r.randint(2, 8)} semaines.",
        f"Contrôle prévu le {_date(r)}. Conseils : {r.choice(['repos', 'alimentation tiède', 'marche quotidienne', 'éviter le froid'])}.",
    ]
    extra = r.randint(0, 3)
    for _ in range(extra):
        paras.append(f"Note de suivi du {_date(r)} : évolution {r.choice(['favorable', 'stable', 'lente', 'mitigée'])}, "
                     f"{r.choice(SYMPTOMS)} {r.choice(['en diminution', 'persistante', 'résolue'])}.")
    return {"doc_id": i + 1, "filename": f"note_{i + 1:05d}.txt", "doc_type": "compte-rendu",
            "patient_id": f"P{r.randint(1, max(2, i // 3 + 1)):05d}", "text": "\n".join(paras)}


def synthetic_notes(n: int = 1000, seed: int = 0) -> list[dict]:
    return [synthetic_note(i, seed) for i in range(n)]


QUESTION_TEMPLATES = [
    "Quelles plantes recommander pour un patient présentant un syndrome « {s} » ?",
    "Le patient souffre de {y}. Quel syndrome évoquer et quelles plantes prescrire ?",
    "Pour {s}, quelle est la plante Empereur et quel est son score de pertinence ?",
    "Quelle formule utiliser en cas de {y} associé à {s} ?",
    "Classe les plantes utiles contre {y} selon leur score.",
    "Quel traitement a été prescrit au patient suivi pour {y} ?",
]


def synthetic_questions(n: int, seed: int = 0) -> list[str]:
    r = _rng(seed + 4242)
    return [r.choice(QUESTION_TEMPLATES).format(s=r.choice(SYNDROMES), y=r.choice(SYMPTOMS))
            for _ in range(n)]


UNIQUE_TEMPLATES = [
    "Patient {pid}, {age} ans, {sex}, consulte pour {y1} et {y2} depuis {w} semaines "
    "(tension {sys}/{dia} mmHg). Quelles plantes recommander pour un syndrome « {s} » ?",
    "Dossier {pid} : {sex} de {age} ans sous {med}, {y1} depuis {w} semaines. "
    "Quel syndrome évoquer et quelle formule prescrire ?",
    "Pour le patient {pid} ({age} ans) présentant {y1}, {y2} et un pouls {pouls}, "
    "quelle est la plante Empereur du syndrome « {s} » et son score ?",
    "Chez {sex_art} de {age} ans (dossier {pid}) traitée par {med}, peut-on associer des plantes "
    "contre {y1} sans interaction ? Syndrome suspecté : « {s} ».",
    "Le patient {pid}, {age} ans, signale {y1} apparue il y a {w} semaines et une langue {langue}. "
    "Classe les plantes utiles selon leur score.",
    "Quel traitement a été prescrit au patient {pid} suivi depuis {w} semaines pour {y1} "
    "et {y2} (contrôle du {date}) ?",
    "Patient {pid} ({sex}, {age} ans, {poids} kg) : {y1} et {y2} malgré {med}. "
    "Quelle posologie de plantes pour « {s} » ?",
    "Résume les plantes Ministre utiles au dossier {pid} : {y1} depuis {w} semaines, "
    "tension {sys}/{dia} mmHg, syndrome « {s} » ({organ}).",
]


def synthetic_unique_questions(n: int, seed: int = 0) -> list[str]:
    """``n`` pairwise-distinct practitioner questions, one per request (the reference
    serves each ``/ask/`` call with a fresh question, llm-qa/main.py:111-117): patient id,
    age, sex, symptom pair, duration, medication and vitals vary per question, so no two
    requests share their question text and retrieval spreads over the corpus.  Collisions
    are redrawn, so every question is distinct."""
    r = _rng(seed + 9091)
    out, seen = [], set()
    while len(out) < n:
        y1, y2 = r.sample(SYMPTOMS, 2)
        fem = r.random() < 0.5
        q = r.choice(UNIQUE_TEMPLATES).format(
            pid=f"P{r.randint(1, 99999):05d}", age=r.randint(18, 92),
            sex="femme" if fem else "homme", sex_art="une femme" if fem else "un homme",
            y1=y1, y2=y2, w=r.randint(1, 52), s=r.choice(SYNDROMES), med=r.choice(MEDS),
            sys=r.randint(95, 175), dia=r.randint(55, 105), poids=r.randint(45, 120),
            pouls=r.choice(["fin", "rapide", "tendu", "faible", "glissant", "profond"]),
            langue=r.choice(["pâle", "rouge", "enduit blanc", "enduit jaune", "violacée"]),
            organ=r.choice(ORGANS), date=_date(r))
        if q not in seen:
            seen.add(q)
            out.append(q)
    return out


def corpus_text(seed: int = 0, n_notes: int = 600) -> list[str]:
    """Text used to train the offline tokenizers."""
    from .kb import base_row_text, matrix_row_text

    m, b = synthetic_kb(seed=seed)
    out = [matrix_row_text(x) for x in m] + [base_row_text(x) for x in b]
    out += [n["text"] for n in synthetic_notes(n_notes, seed)]
    out += synthetic_questions(400, seed)
    return out
