"""Prompt templates of the generator-facing services.

* ``REFERENCE_QA_TEMPLATE`` -- the reference llm-qa "stuff" prompt, character for
  character (llm-qa/main.py:71-93): the retrieved context comes FIRST, then the
  instructions and the practitioner question.
* ``CACHE_FRIENDLY_QA_TEMPLATE`` -- the same slots and instructions with every fixed
  line moved in front of ``{context}``, so all requests share a long token prefix that
  the engine's prefix cache serves from HBM (with the reference order, prompts diverge
  after ~60 tokens).  Opt-in with ``QA_TEMPLATE=cache_friendly``; the llm-qa service
  asks the verbatim reference text by default, as the reference does (``qa_template``).
  ``bench.py`` names the template it measures in its JSON line (``workload.template``).
* ``SINGLE_PATIENT_TEMPLATE`` / ``MULTI_PATIENT_TEMPLATE`` -- the synthese-comparative
  templates, verbatim (synthese-comparative/core/prompts.py:3-45); the synthese service
  uses them as they are.

The verbatim texts are API-visible behaviour (what the LLM is asked), so they are kept
byte-identical; ``tests/test_ui_and_prompts_cpu.py`` compares them with the reference
files when those are mounted.
"""
from __future__ import annotations

import os

REFERENCE_QA_TEMPLATE = (
    "\n"
    "Tu es un Expert en Pharmacopée Chinoise (MTC).\n"
    "Tu disposes d'extraits de ta base de données contenant des SCORES DE PERTINENCE pour chaque plante.\n"
    "\n"
    "CONTEXTE (Données MTC + Dossier Patient) :\n"
    "{context}\n"
    "\n"
    "INSTRUCTIONS STRICTES :\n"
    "1. ANALYSE : Identifie le syndrome du patient dans le contexte.\n"
    "2. RECHERCHE : Trouve dans le contexte les plantes associées à ce syndrome.\n"
    "3. CLASSEMENT : Trie les plantes selon leur \"Score de pertinence\" (indiqué dans le contexte).\n"
    "   - Score 10 = Plante Empereur (Indispensable)\n"
    "   - Score 7 = Plante Ministre\n"
    "4. RÉPONSE :\n"
    "   - Présente ta réponse sous forme de liste priorisée.\n"
    "   - Mentionne toujours le Score et le Rôle pour justifier ton choix.\n"
    "   - Exemple : \"1. [Plante] (Score 10, Empereur) : Recommandée car...\"\n"
    "\n"
    "QUESTION DU PRATICIEN : \n"
    "{question}\n"
    "\n"
    "RÉPONSE EXPERT :\n"
)

# Expert-assistant prompt with the same slots as the reference's QA_CHAIN_PROMPT
# (instructions, context block, practitioner question).  All fixed text comes FIRST so
# every request shares a long token prefix: the engine's prefix cache then serves those
# KV blocks from HBM instead of recomputing them.
CACHE_FRIENDLY_QA_TEMPLATE = """Vous êtes un expert en pharmacopée chinoise (MTC) assistant un praticien.
Vous recevez des extraits de la base de connaissances et des dossiers patients ; chaque
plante y est accompagnée d'un score de pertinence.

CONSIGNES :
1. Repérez le syndrome du patient dans les extraits.
2. Relevez les plantes associées à ce syndrome.
3. Ordonnez-les par score de pertinence décroissant (10 = plante Empereur, 7 = plante Ministre).
4. Répondez par une liste numérotée en justifiant chaque plante par son score et son rôle,
   par exemple : "1. [Plante] (score 10, Empereur) : recommandée parce que ...".
5. N'utilisez que les informations des extraits ; si elles sont insuffisantes, dites-le.

EXTRAITS (base MTC et dossier patient) :
{context}

QUESTION DU PRATICIEN :
{question}

RÉPONSE DE L'EXPERT :
"""

QA_TEMPLATES = {"reference": REFERENCE_QA_TEMPLATE, "cache_friendly": CACHE_FRIENDLY_QA_TEMPLATE}


DEFAULT_QA_TEMPLATE = "reference"


def qa_template(name: str | None = None) -> str:
    """The QA prompt template named ``name`` (default: env ``QA_TEMPLATE``, else the
    verbatim reference prompt)."""
    name = name or os.environ.get("QA_TEMPLATE", DEFAULT_QA_TEMPLATE)
    try:
        return QA_TEMPLATES[name]
    except KeyError:
        raise ValueError(f"QA_TEMPLATE must be one of {sorted(QA_TEMPLATES)}, got {name!r}") from None


SINGLE_PATIENT_TEMPLATE = """
You are a medical assistant. Summarize the following clinical history
for ONE anonymized patient.

Context:
- Patient alias: {patient_alias}
- Time window: {from_date} to {to_date}
- Clinical focus: {focus}

Clinical notes:
{documents}

Task:
Produce a structured summary in FRENCH with sections:
1. Contexte général
2. Focus clinique ({focus})
3. Événements clés
4. Points de vigilance

Return ONLY the summary text (no extra comments, no JSON).
"""


MULTI_PATIENT_TEMPLATE = """
You are a medical assistant. Compare the clinical histories of
MULTIPLE anonymized patients.

Context:
- Patient aliases: {patients}
- Time window: {from_date} to {to_date}
- Clinical focus: {focus}

Clinical notes by patient:
{documents_by_patient}

Task:
In FRENCH, produce:
1. A global comparative summary
2. The main differences between patients (by dimensions: traitement, événements, risques...)
3. The key risk points for each patient

Return ONLY the final text (no extra comments, no JSON).
"""
